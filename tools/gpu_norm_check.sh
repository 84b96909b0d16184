#!/bin/bash
# norm backward with per-block partial rows: model / config / determinism tests, then the bench.
cd $GRAFT_REPO_ROOT
out=gpurun_out/norm; mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_determinism_gpu.py tests/test_configs_gpu.py > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
timeout -k 10 600 python -u bench.py --no-roofline --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 4; }
cut -c1-300 $out/bench.json
