"""Shared pytest setup: markers, import paths, golden-fixture loader."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(ROOT, "mamba-clip_amd")
for p in (ROOT, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")


def load_golden(name):
    from safetensors.torch import load_file
    return load_file(os.path.join(GOLDEN, name))


def golden_meta(name):
    from safetensors import safe_open
    with safe_open(os.path.join(GOLDEN, name), framework="pt") as f:
        return f.metadata() or {}


@pytest.fixture
def golden():
    return load_golden


@pytest.fixture(autouse=True)
def _restore_tf32_flags():
    """init_device (utils/dist_utils.py, as the reference's) turns TF32 on process-wide; tests that
    run it (CLI, train) must not change the precision of fp32 reference matmuls in later tests."""
    import torch
    saved = (torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32)
    yield
    torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = saved
