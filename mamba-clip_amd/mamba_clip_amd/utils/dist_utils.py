"""Process-group bring-up (reference: src/mamba_clip/utils/dist_utils.py:9-123).

One process per GPU.  torch.distributed backend "nccl" is RCCL on ROCm (feature
all-gather + DDP gradient all-reduce over xGMI); "gloo" for CPU tests.  Fixes
the reference's torchrun path (datetime.timedelta
AttributeError, rank read before the env).
"""
import os
from datetime import timedelta

import torch
import torch.distributed as dist


def world_info_from_env():
    local_rank = 0
    for v in ("LOCAL_RANK", "MPI_LOCALRANKID", "SLURM_LOCALID", "OMPI_COMM_WORLD_LOCAL_RANK"):
        if v in os.environ:
            local_rank = int(os.environ[v])
            break
    global_rank = 0
    for v in ("RANK", "PMI_RANK", "SLURM_PROCID", "OMPI_COMM_WORLD_RANK"):
        if v in os.environ:
            global_rank = int(os.environ[v])
            break
    world_size = 1
    for v in ("WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS", "OMPI_COMM_WORLD_SIZE"):
        if v in os.environ:
            world_size = int(os.environ[v])
            break
    return local_rank, global_rank, world_size


def is_using_distributed():
    if "WORLD_SIZE" in os.environ:
        return int(os.environ["WORLD_SIZE"]) > 1
    if "SLURM_NTASKS" in os.environ:
        return int(os.environ["SLURM_NTASKS"]) > 1
    return False


def init_device(args):
    """Sets args.distributed / world_size / rank / local_rank / device; returns the torch.device."""
    args.distributed = False
    args.world_size = 1
    args.rank = 0
    args.local_rank = 0
    if is_using_distributed():
        args.local_rank, args.rank, args.world_size = world_info_from_env()
        backend = getattr(args, "dist_backend", "nccl")
        if backend == "nccl" and not torch.cuda.is_available():
            backend = "gloo"
        if torch.cuda.is_available():
            torch.cuda.set_device(args.local_rank)
        dist.init_process_group(backend=backend, init_method=getattr(args, "dist_url", "env://"),
                                world_size=args.world_size, rank=args.rank, timeout=timedelta(seconds=3600))
        args.distributed = True
    if torch.cuda.is_available():
        device = torch.device(f"cuda:{args.local_rank}")
        torch.cuda.set_device(device)
        torch.backends.cuda.matmul.allow_tf32 = True
        torch.backends.cudnn.allow_tf32 = True
    else:
        device = torch.device("cpu")
    args.device = str(device)
    return device


def broadcast_object(args, obj, src=0):
    if getattr(args, "distributed", False):
        objects = [obj if args.rank == src else None]
        dist.broadcast_object_list(objects, src=src)
        return objects[0]
    return obj


def is_global_master(args):
    return getattr(args, "rank", 0) == 0


def is_local_master(args):
    return getattr(args, "local_rank", 0) == 0


def is_master(args, local=False):
    return is_local_master(args) if local else is_global_master(args)
