set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stream_audit.py --out gpurun_out/i_audit_image.json > gpurun_out/i_audit_image.log 2>&1; echo "audit image rc=$?"
timeout -k 10 300 python -u tools/stream_audit.py --side-tower text --out gpurun_out/i_audit_text.json > gpurun_out/i_audit_text.log 2>&1; echo "audit text rc=$?"
echo done
