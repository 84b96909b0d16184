#!/bin/bash
# Round-4 check 24: x_proj gradient slab (dB / dC and d(dt_raw) written in place) -- tests, C2 A/B
set -u
out=gpurun_out/r04c24; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_scan_gpu.py tests/test_configs_gpu.py tests/test_abi.py > $out/pytest.txt 2>&1 || { echo pytest failed; tail -60 $out/pytest.txt; exit 2; }
tail -3 $out/pytest.txt
for t in 1 0 1 0; do
  MAMBA_CLIP_AMD_XPROJ_GRAD_SLAB=$t timeout -k 10 300 python bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c2_$t.json 2> $out/c2_$t.err || { echo c2 failed; tail -20 $out/c2_$t.err; exit 3; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('c2 xproj_slab', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'], r['final_loss'])" $out/c2_$t.json $t | tee -a $out/summary.txt
done
