set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 3 --repeats 10"
timeout -k 10 400 $P --variants conc,conc_image > gpurun_out/al_c2.log 2>&1; echo "c2 rc=$?"; grep '"runs"' gpurun_out/al_c2.log | cut -c1-420
timeout -k 10 400 $P --model biomedclip-vit_b16-pubmedbert256 --batch 64 --variants conc > gpurun_out/al_c3.log 2>&1; echo "c3 rc=$?"; grep '"runs"' gpurun_out/al_c3.log | cut -c1-420
timeout -k 10 400 $P --batch 32 --variants conc,conc_image > gpurun_out/al_c2b32.log 2>&1; echo "c2 b32 rc=$?"; grep '"runs"' gpurun_out/al_c2b32.log | cut -c1-420
B="python -u bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline"
timeout -k 10 300 $B > gpurun_out/al_b_text.log 2>&1 && echo "c2 text-side: $(tail -1 gpurun_out/al_b_text.log | cut -c1-150)"
MAMBA_CLIP_AMD_SIDE_TOWER=image timeout -k 10 300 $B > gpurun_out/al_b_img.log 2>&1 && echo "c2 image-side: $(tail -1 gpurun_out/al_b_img.log | cut -c1-150)"
timeout -k 10 300 $B > gpurun_out/al_b_text2.log 2>&1 && echo "c2 text-side: $(tail -1 gpurun_out/al_b_text2.log | cut -c1-150)"
echo done
