set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 3 --repeats 10"
timeout -k 10 300 $P --batch 32 --variants conc,conc_image > gpurun_out/ar_b32.log 2>&1; echo "b32: $(grep '"runs"' gpurun_out/ar_b32.log | cut -c1-200)"
timeout -k 10 300 $P --variants conc,conc_image > gpurun_out/ar_b256.log 2>&1; echo "b256: $(grep '"runs"' gpurun_out/ar_b256.log | cut -c1-200)"
timeout -k 10 300 $P --model biomedclip-vit_b16-pubmedbert256 --batch 64 --variants conc > gpurun_out/ar_c3.log 2>&1; echo "c3: $(grep '"runs"' gpurun_out/ar_c3.log | cut -c1-200)"
B="python -u bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline"
for j in 1 0 1 0; do
  MAMBA_CLIP_AMD_SCAN_BWD_JOIN=$j timeout -k 10 300 $B > gpurun_out/ar_bench_$j.log 2>&1 && echo "join=$j: $(tail -1 gpurun_out/ar_bench_$j.log | cut -c90-160)"
done
echo done
