"""Time the config-5 fp8 similarity leg of bench.py on its own (for rocprofv3 runs)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

from mamba_clip_amd import _lib  # noqa: E402

_lib.load()
print(json.dumps(bench.similarity_c5()), flush=True)
