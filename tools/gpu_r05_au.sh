set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_step.py --toggle ops.WGRAD_HIP --steps 10 --reps 4 > gpurun_out/au_ab_c2.log 2>&1; echo "ab c2 rc=$?"; grep "rep " gpurun_out/au_ab_c2.log
timeout -k 10 300 python -u tools/ab_step.py --toggle ops.WGRAD_HIP --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 10 --reps 4 > gpurun_out/au_ab_c3.log 2>&1; echo "ab c3 rc=$?"; grep "rep " gpurun_out/au_ab_c3.log
echo done
