set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/stress_determinism.py --iters 40 --ops gemm_in_proj,gemm_out_dgrad,bmm_f32 --loads none,gemm,gemm_vit,attn > gpurun_out/stress_gemm.log 2>&1; echo "stress tuned rc=$?"
STRESS_TUNED=0 timeout -k 10 400 python -u tools/stress_determinism.py --iters 40 --ops gemm_in_proj,gemm_out_dgrad,bmm_f32 --loads none,gemm_vit > gpurun_out/stress_gemm_untuned.log 2>&1; echo "stress untuned rc=$?"
echo done
