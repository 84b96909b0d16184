#!/bin/bash
# Round 6 GPU batch D: eager vs two-stream / one-stream HIP-graph C2 step (bench.py), interleaved.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06_d
for rep in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > gpurun_out/r06_d/eager_$rep.json 2> gpurun_out/r06_d/eager_$rep.err || exit 1
  timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline --graph 1 > gpurun_out/r06_d/graph2_$rep.json 2> gpurun_out/r06_d/graph2_$rep.err || exit 1
done
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline --graph 1 --graph-streams 1 > gpurun_out/r06_d/graph1.json 2> gpurun_out/r06_d/graph1.err || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_scan_gpu.py > gpurun_out/r06_d/scan.log 2>&1 || exit 1
L=mamba-clip_amd/mamba_clip_amd
for v in sel1 prod; do
  so=$PWD/$L/libmamba_clip_amd.so; [ $v != prod ] && so=$PWD/$L/libmamba_clip_amd_v_$v.so
  for rep in 1 2; do
    for f in "" "--train-fwd"; do
      MAMBA_CLIP_AMD_LIB=$so timeout -k 10 120 python3 -u tools/time_scan.py --shape 64,3072,4096,16 $f --iters 10 \
        >> gpurun_out/r06_d/c4_fwd_$v.log 2>&1 || exit 1
    done
  done
done
