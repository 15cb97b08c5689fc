cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
(cd /tmp && timeout -k 10 60 rocprofv3 --list-avail > "$GRAFT_REPO_ROOT/gpurun_out/avail.txt" 2>&1); echo "list rc=$?"
grep -i -o "SQ_[A-Z_]*MFMA[A-Z0-9_]*\|GRBM_GUI_ACTIVE" gpurun_out/avail.txt | sort -u | head -30
bash scripts/gpu_pmc.sh
