#!/bin/bash
# Round-4 check 2: gradient checkpointing on the GPU; the exp2-polynomial A/B of the forward
# recurrence (parity of the variant + interleaved C4 timing); PMC traffic of the shipped forward.
set -u
out=gpurun_out/r04c2; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    "tests/test_model_gpu.py::test_grad_checkpointing_bitwise_gpu" > $out/pytest_ckpt.log 2>&1 \
    || { echo ckpt tests failed; tail -30 $out/pytest_ckpt.log; exit 1; }
tail -1 $out/pytest_ckpt.log
MAMBA_CLIP_AMD_LIB=ab_libs/lib_poly1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_scan_gpu.py > $out/pytest_poly1.log 2>&1 \
    || { echo poly1 scan tests failed; tail -30 $out/pytest_poly1.log; exit 2; }
tail -1 $out/pytest_poly1.log
for rep in 1 2 3; do
  for v in base poly1 poly2; do
    if [ $v = base ]; then lib=""; else lib=ab_libs/lib_$v.so; fi
    r=$(MAMBA_CLIP_AMD_LIB=$lib timeout -k 5 90 python tools/time_scan.py --iters 20 2>&1 | grep -o "[0-9.]* ms" | head -1) || exit 3
    echo "rep $rep $v C4 fwd $r" | tee -a $out/poly_ab.txt
  done
done
bash tools/pmc_traffic.sh $out/pmc > $out/pmc.log 2>&1 || { echo pmc failed; tail -20 $out/pmc.log; exit 4; }
tail -25 $out/pmc.log
