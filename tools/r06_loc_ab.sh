#!/bin/bash
# Round 6 localisation A/B: in-step vs solo layer-23 scan backward under library / env variants.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06_loc
L=mamba-clip_amd/mamba_clip_amd
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 150 python3 -u tools/scan_bwd_localize.py --batch 32 --runs ${RUNS:-5} > gpurun_out/r06_loc/g_$n.log 2>&1 || exit 1
}
for v in ${VARIANTS:-permnop nogemm nowgrad}; do
  case $v in
    permnop) run permnop MAMBA_CLIP_AMD_LIB=$PWD/$L/libmamba_clip_amd_v_permnop.so ;;
    nogemm) run nogemm MAMBA_CLIP_AMD_WGRAD_HIP=0 MAMBA_CLIP_AMD_MLP_HIP_FC2=0 MAMBA_CLIP_AMD_MLP_HIP_BWD=0 MAMBA_CLIP_AMD_SMALL_K_HIP=0 ;;
    nowgrad) run nowgrad MAMBA_CLIP_AMD_WGRAD_HIP=0 ;;
    nomlp) run nomlp MAMBA_CLIP_AMD_MLP_HIP_FC2=0 MAMBA_CLIP_AMD_MLP_HIP_BWD=0 ;;
    dbg) env MAMBA_CLIP_AMD_LIB=$PWD/$L/libmamba_clip_amd_v_dbg.so timeout -k 10 150 python3 -u tools/scan_bwd_localize.py --batch 32 --runs ${RUNS:-5} --debug > gpurun_out/r06_loc/g_dbg.log 2>&1 || exit 1 ;;
    *) run $v MAMBA_CLIP_AMD_LIB=$PWD/$L/libmamba_clip_amd_v_$v.so ;;
  esac
done
