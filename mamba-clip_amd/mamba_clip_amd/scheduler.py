"""Learning-rate schedules with warmup restarts (reference: src/mamba_clip/scheduler.py:9-103).

Each factory returns `adjust(step) -> lr` that writes lr into every param group;
train_one_epoch calls it once per optimizer step (train.py:127-128).
"""
import math


def assign_learning_rate(optimizer, new_lr):
    for group in optimizer.param_groups:
        group["lr"] = new_lr


def _warmup(base_lr, warmup_length, step):
    return base_lr * (step + 1) / warmup_length


def _cycle(step, restart_interval):
    return step % restart_interval if restart_interval else step


def const_lr(optimizer, base_lr, warmup_length, total_steps, restart_interval=None):
    def adjust(step):
        s = _cycle(step, restart_interval)
        lr = _warmup(base_lr, warmup_length, s) if s < warmup_length else base_lr
        assign_learning_rate(optimizer, lr)
        return lr
    return adjust


def const_lr_cooldown(optimizer, base_lr, warmup_length, total_steps, cooldown_steps, restart_interval=None,
                      cooldown_power=1.0, cooldown_end_lr=0.0):
    def adjust(step):
        s = _cycle(step, restart_interval)
        period = restart_interval if restart_interval else total_steps
        start = period - cooldown_steps
        if s < warmup_length:
            lr = _warmup(base_lr, warmup_length, s)
        elif s < start:
            lr = base_lr
        else:
            decay = (1 - (s - start) / (period - start)) ** cooldown_power
            lr = decay * (base_lr - cooldown_end_lr) + cooldown_end_lr
        assign_learning_rate(optimizer, lr)
        return lr
    return adjust


def cosine_lr(optimizer, base_lr, warmup_length, total_steps, restart_interval=None):
    def adjust(step):
        s = _cycle(step, restart_interval)
        if s < warmup_length:
            lr = _warmup(base_lr, warmup_length, s)
        else:
            period = (restart_interval if restart_interval else total_steps) - warmup_length
            lr = 0.5 * (1 + math.cos(math.pi * (s - warmup_length) / period)) * base_lr
        assign_learning_rate(optimizer, lr)
        return lr
    return adjust
