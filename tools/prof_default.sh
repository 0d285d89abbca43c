# The exact default bench command under rocprofv3 --kernel-trace --stats (its
# hipEvent kernel averages must agree with rocprof's), then the round profile
# (200-epoch trace + FETCH/WRITE/MFMA PMC passes).  usage: tools/prof_default.sh <tag>
set -u
R="$GRAFT_REPO_ROOT"; tag="${1:-r02}"; export TMPDIR=/tmp
out="$R/gpurun_out/prof_default_$tag"; mkdir -p "$out"
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 "$R/bench.py" > "$out/bench.log" 2>&1 || { echo "trace rc=$?"; tail "$out/bench.log"; exit 1; }
find "$out/trace" -name '*kernel_stats.csv' -exec cp {} "$out/kernel_stats.csv" \;
tail -1 "$out/bench.log" | cut -c1-600
cd "$R" && bash tools/profile_round.sh "$tag" bf16x3
