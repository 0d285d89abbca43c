set -u
R="$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p "$R/gpurun_out/prof_default"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_default/trace" -o run --output-format csv -- python3 "$R/bench.py" > "$R/gpurun_out/prof_default/bench.log" 2>&1 || { echo "trace rc=$?"; tail "$R/gpurun_out/prof_default/bench.log"; exit 1; }
find "$R/gpurun_out/prof_default/trace" -name '*kernel_stats.csv' -exec cp {} "$R/gpurun_out/prof_default/kernel_stats.csv" \;
tail -1 "$R/gpurun_out/prof_default/bench.log" | cut -c1-400
cd "$R" && bash tools/profile_round.sh x3q bf16x3
