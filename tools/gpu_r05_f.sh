set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u tools/determinism_probe.py --compare prev --steps 2 --repeats 6 --variants conc,conc_sharedcast,seq --out gpurun_out/det3.json > gpurun_out/det3.log 2>&1; echo "det3 rc=$?"
timeout -k 10 300 python -u tools/ab_step.py --toggle ops.WGRAD_HIP --steps 10 --reps 3 > gpurun_out/ab_wgrad_c2.log 2>&1; echo "ab c2 rc=$?"
timeout -k 10 300 python -u tools/ab_step.py --toggle ops.WGRAD_HIP --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 10 --reps 3 > gpurun_out/ab_wgrad_c3.log 2>&1; echo "ab c3 rc=$?"
echo done
