#!/bin/bash
# Round-4 check 33: C3 side-stream arrangement (text high = default, image normal, image high); GPU tests of the
# two-stream paths with the new C2 default (image tower on the side stream)
set -u
out=gpurun_out/r04c33; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_dist_gloo.py tests/test_graph_gpu.py > $out/pytest.txt 2>&1 || { echo pytest failed; tail -40 $out/pytest.txt; exit 2; }
tail -2 $out/pytest.txt
for v in "text -1" "image 0" "image -1" "text -1" "image 0" "image -1"; do
  set -- $v
  MAMBA_CLIP_AMD_SIDE_TOWER=$1 MAMBA_CLIP_AMD_SIDE_PRIORITY=$2 timeout -k 10 300 python bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c3_$1_$2.json 2> $out/c3_$1_$2.err || { echo c3 failed; tail -20 $out/c3_$1_$2.err; exit 3; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('c3 side', sys.argv[2], 'prio', sys.argv[3], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'], r['final_loss'])" $out/c3_$1_$2.json $1 $2 | tee -a $out/summary.txt
done
