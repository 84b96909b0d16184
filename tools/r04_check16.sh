#!/bin/bash
set -u
out=gpurun_out/r04c16; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_configs_gpu.py -k "bf16_autocast or 790m" > $out/pytest.txt 2>&1 || { echo pytest failed; tail -50 $out/pytest.txt; exit 2; }
grep -E "bf16 mixer|790M layer|passed|failed" $out/pytest.txt
