set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline"
for q in 4 1 4 1; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 $B > gpurun_out/r_bench_c2_q$q.log 2>&1 || { echo "bench c2 q$q failed"; exit 1; }
  echo "c2 q$q: $(tail -1 gpurun_out/r_bench_c2_q$q.log | cut -c1-160)"
done
for q in 4 1; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 $B --model biomedclip-vit_b16-pubmedbert256 --batch 64 > gpurun_out/r_bench_c3_q$q.log 2>&1 || { echo "bench c3 q$q failed"; exit 1; }
  echo "c3 q$q: $(tail -1 gpurun_out/r_bench_c3_q$q.log | cut -c1-160)"
done
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python -u tools/determinism_probe.py --summary --self-ref --steps 3 --repeats 10 --variants conc,conc_text > gpurun_out/r_det_q1.log 2>&1; echo "det q1 c2"; grep '"runs"' gpurun_out/r_det_q1.log
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python -u tools/determinism_probe.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --summary --self-ref --steps 3 --repeats 10 --variants conc > gpurun_out/r_det_q1_c3.log 2>&1; echo "det q1 c3"; grep '"runs"' gpurun_out/r_det_q1_c3.log
timeout -k 10 300 python -u tools/determinism_probe.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --summary --self-ref --steps 3 --repeats 10 --variants conc > gpurun_out/r_det_q4_c3.log 2>&1; echo "det q4 c3"; grep '"runs"' gpurun_out/r_det_q4_c3.log
echo done
