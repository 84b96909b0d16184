set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/stress_determinism.py --iters 40 --ops sum0,sum_cls,colsum_f32,scan_bwd --loads none,scan,scan_nofine,scan_fwd,gemm_vit > gpurun_out/w_stress.log 2>&1; echo "stress rc=$?"
grep '"op"' gpurun_out/w_stress.log
echo done
