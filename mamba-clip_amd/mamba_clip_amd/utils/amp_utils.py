"""Precision policy (reference: src/mamba_clip/utils/amp_utils.py:19-52).

amp -> fp16 autocast (+GradScaler); amp_bf16 / amp_bfloat16 -> bf16 autocast;
bf16 / pure_bf16 / fp16 / pure_fp16 -> input dtype; anything else -> fp32.
"""
from contextlib import suppress

import torch

PRECISION_AMP = "amp"
PRECISION_AMP_BFLOAT16 = "amp_bfloat16"
PRECISION_AMP_BF16 = "amp_bf16"
PRECISION_BFLOAT16_OPTIONS = {"bf16", "pure_bf16"}
PRECISION_FLOAT16_OPTIONS = {"fp16", "pure_fp16"}


def get_autocast(precision):
    if precision == PRECISION_AMP:
        return lambda: torch.autocast("cuda", dtype=torch.float16)
    if precision in {PRECISION_AMP_BFLOAT16, PRECISION_AMP_BF16}:
        return lambda: torch.autocast("cuda", dtype=torch.bfloat16)
    return suppress


def get_input_dtype(precision):
    if precision in PRECISION_BFLOAT16_OPTIONS:
        return torch.bfloat16
    if precision in PRECISION_FLOAT16_OPTIONS:
        return torch.float16
    return None
