#!/bin/bash
# Round-4 check 1: scan forward without the B/C pre-pass (parity + time), two-stream towers beside a
# BERT tower (C3) with data-parallel GEMM grids, concurrent stream-K probe, C2 / C3 bench lines.
set -u
out=gpurun_out/r04c1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_scan_gpu.py \
    tests/test_configs_gpu.py "tests/test_model_gpu.py::test_concurrent_towers_bitwise_identical" \
    tests/test_dist_gloo.py -m gpu > $out/pytest.log 2>&1 || { echo pytest failed; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 120 python tools/time_scan.py --iters 30 > $out/c4_fwd.txt 2>&1 || { echo time_scan failed; cat $out/c4_fwd.txt; exit 2; }
cat $out/c4_fwd.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/c3conc -o k -- \
    python tools/sk_probe.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --concurrent --out $out/c3conc.json \
    > $out/c3conc.log 2>&1 || { echo c3 concurrent probe failed; tail -20 $out/c3conc.log; exit 3; }
python tools/sk_probe_report.py $(ls $out/c3conc/*kernel_trace.csv | head -1) $out/c3conc.json > $out/c3conc.txt; tail -1 $out/c3conc.txt
timeout -k 10 300 python bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 30 --warmup 5 \
    --no-cpu-baseline --no-roofline > $out/bench_c3.json 2> $out/bench_c3.err || { echo c3 bench failed; tail -20 $out/bench_c3.err; exit 4; }
cut -c1-250 $out/bench_c3.json
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err || { echo c2 bench failed; tail -20 $out/bench_c2.err; exit 5; }
cut -c1-600 $out/bench_c2.json
