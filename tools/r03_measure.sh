#!/bin/bash
# Round-3 measurement pass: rocprofv3 kernel-trace summary of the default bench command (the roofline
# kernel's average duration must agree with the bench's HIP-event figure), then the C3 bench line.
set -u
out=gpurun_out/r03m; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/bench_trace -o b -- python bench.py --steps 10 --warmup 5 > $out/bench_traced.json 2> $out/bench_traced.err || { echo traced bench failed; tail -20 $out/bench_traced.err; exit 1; }
tail -1 $out/bench_traced.json | cut -c1-400
grep -E "scan_fwd_pair|bc_relayout|sim_fp8|attn_" $out/bench_trace/b_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 400 python bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $out/bench_c3.json 2> $out/bench_c3.err || { echo c3 failed; tail -20 $out/bench_c3.err; exit 2; }
cut -c1-300 $out/bench_c3.json
