set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --steps 2"
timeout -k 10 300 $P --repeats 12 --variants seq,conc,conc_sync,conc_fsync,conc_text,conc_nofine,conc_noattn,conc_nowt,conc_torchadam --out gpurun_out/h_det.json > gpurun_out/h_det.log 2>&1; echo "det rc=$?"
PYTORCH_NO_CUDA_MEMORY_CACHING=1 timeout -k 10 300 $P --repeats 12 --variants seq,conc,conc_sync --out gpurun_out/h_det_nocache.json > gpurun_out/h_det_nocache.log 2>&1; echo "det nocache rc=$?"
timeout -k 10 300 $P --fill-nan --repeats 6 --variants seq,conc > gpurun_out/h_det_nan.log 2>&1; echo "det nan rc=$?"
timeout -k 10 300 python -u tools/stress_determinism.py --iters 30 --ops gemm_in_proj,gemm_out_dgrad,bmm_f32,scan_bwd,rms_bwd,conv_bwd --loads none,gemm_vit,attn > gpurun_out/h_stress.log 2>&1; echo "stress rc=$?"
echo done
