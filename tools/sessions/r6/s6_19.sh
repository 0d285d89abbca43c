#!/usr/bin/env bash
# round 6: profiles of the current library — the isolated deep W = 256
# chunk-epoch (kernel trace + FETCH/WRITE/MFMA-busy passes, rows and params),
# then the default bench under rocprofv3 --kernel-trace --stats
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
bash tools/r4/iso_prof.sh r6b 256 rows > gpurun_out/iso_prof_r6b.log 2>&1 || { echo "iso_prof rc=$?"; tail -20 gpurun_out/iso_prof_r6b.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/iso_r6b/summary.json'))
for k,v in d.items(): print(k, {x: v[x] for x in ('bytes','mfma_busy','rocprof_avg_ms','hipevent_avg_ms','rocprof_vs_hipevent','lib_sha16')})"
export TMPDIR=/tmp
out="$R/gpurun_out/prof_bench_r6"; mkdir -p "$out"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 "$R/bench.py" > "$out/bench.log" 2> "$out/bench.err" || { echo "bench trace rc=$?"; tail "$out/bench.err"; exit 1; }
find "$out/trace" -name '*kernel_stats.csv' -exec cp {} "$out/kernel_stats.csv" \;
rm -rf "$out/trace"
grep '^{' "$out/bench.log" | cut -c1-200
