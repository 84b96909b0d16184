set -e
mkdir -p gpurun_out/diag
for t in main nored noexp none; do
  if [ $t = main ]; then lib=mamba-clip_amd/mamba_clip_amd/libmamba_clip_amd.so; else lib=mamba-clip_amd/mamba_clip_amd/libmamba_clip_amd_diag_$t.so; fi
  MAMBA_CLIP_AMD_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/diag/$t -o t --output-format csv -- python tools/time_scan.py --shape 256,1536,80,16 --iters 5 --bwd > gpurun_out/diag/$t.log 2>&1
done
