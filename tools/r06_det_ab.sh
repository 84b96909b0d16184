#!/bin/bash
# Round 6: is the two-stream C2 step's run-to-run divergence an inline-asm hazard in the scan kernels?
# Same determinism probe (default hardware queues, towers on two streams, batch 32: 10 of 10 runs differed
# in round 5) against three builds of the library:
#   base  -- the round-5 tree
#   fix   -- v_permlane*_swap operands of the backward's channel reduction behind >= 2 wait states
#   audit -- fix + every arithmetic asm block of the scan kernels followed by s_nop 4
# Output: gpurun_out/r06_det/<lib>.log (one JSON summary line per variant).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06_det
mkdir -p $OUT
B=${B:-32}
REP=${REP:-8}
LIBS=${LIBS:-"base fix audit"}
for lib in $LIBS; do
  case $lib in
    base) so=mamba-clip_amd/mamba_clip_amd/libmamba_clip_amd_base.so ;;
    fix) so=mamba-clip_amd/mamba_clip_amd/libmamba_clip_amd.so ;;
    audit) so=mamba-clip_amd/mamba_clip_amd/libmamba_clip_amd_audit.so ;;
  esac
  echo "== $lib $so" | tee -a $OUT/$lib.log
  MAMBA_CLIP_AMD_LIB=$PWD/$so timeout -k 10 300 python3 -u tools/determinism_probe.py --summary --self-ref \
      --variants conc --batch $B --repeats $REP --steps 2 >> $OUT/$lib.log 2>&1
  rc=$?
  echo "rc $rc" >> $OUT/$lib.log
  tail -3 $OUT/$lib.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
