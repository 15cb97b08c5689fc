cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for px in 4 1 2; do
rm -rf gpurun_out/prof_px$px
(cd /tmp && PGDIST_STEM_PX=$px timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_px$px" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 3 > "$R/gpurun_out/prof_px$px.log" 2>&1) || exit 6
done
