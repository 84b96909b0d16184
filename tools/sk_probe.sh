#!/bin/bash
# Stream-K probe: kernel <-> GEMM shape/tower map for one C2 and one C3 training
# step, default hipBLASLt/rocBLAS grids vs TENSILE_STREAMK_DATA_PARALLEL=1.  Single stream only.
# The package sets the variable to 1 at import unless it is already set, so the default legs export
# 0 explicitly; sk_probe.py records the value it ran with and sk_probe_report.py flags a mismatch.
set -u
out=gpurun_out/skp; mkdir -p $out
export TMPDIR=/tmp
run() {   # tag, env assignment (or "-"), model, batch
  local tag=$1 envs=$2 model=$3 batch=$4
  if [ "$envs" != "-" ]; then export $envs; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/$tag -o k -- \
      python tools/sk_probe.py --model $model --batch $batch --out $out/$tag.json > $out/$tag.log 2>&1 \
      || { echo "$tag failed"; tail -20 $out/$tag.log; exit 1; }
  if [ "$envs" != "-" ]; then unset ${envs%%=*}; fi
  python tools/sk_probe_report.py $(ls $out/$tag/*kernel_trace.csv | head -1) $out/$tag.json > $out/$tag.txt
  tail -1 $out/$tag.txt
}
run c2_default TENSILE_STREAMK_DATA_PARALLEL=0 vit_b16-mamba130m 256
run c2_dp TENSILE_STREAMK_DATA_PARALLEL=1 vit_b16-mamba130m 256
run c3_default TENSILE_STREAMK_DATA_PARALLEL=0 biomedclip-vit_b16-pubmedbert256 64
run c3_dp TENSILE_STREAMK_DATA_PARALLEL=1 biomedclip-vit_b16-pubmedbert256 64
