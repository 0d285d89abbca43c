#!/usr/bin/env bash
# Isolated-leg profile of the dominant kernel:
#  1. rocprofv3 --kernel-trace --stats of tools/r4/isokernel.py (the bench's
#     isolated leg alone): its k_step_rows<256,128>[bf16x3] average must match
#     the hipEvent avg_launch_ms the same run prints (and bench.py reports);
#  2. PMC passes of the same command, one block each: FETCH_SIZE; WRITE_SIZE;
#     SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE.
# usage: tools/r4/iso_prof.sh <tag> [width] [kernel]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
tag="${1:-iso}"; W="${2:-256}"; K="${3:-rows}"
export TMPDIR=/tmp
out="$R/gpurun_out/iso_$tag"; mkdir -p "$out"
cmd=(python3 "$R/tools/r4/isokernel.py" --width "$W" --kernel "$K")
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- "${cmd[@]}" > "$out/trace.log" 2>&1 || { echo "trace rc=$?"; tail -5 "$out/trace.log"; exit 1; }
find "$out/trace" -name '*kernel_stats.csv' -exec cp {} "$out/kernel_stats.csv" \;
tail -1 "$out/trace.log"
i=0
for cs in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $cs -d "$out/p$i" -o run --output-format csv -- "${cmd[@]}" > "$out/p$i.log" 2>&1 || { echo "pmc pass $i rc=$?"; tail -5 "$out/p$i.log"; exit 1; }
  find "$out/p$i" -name '*counter_collection.csv' -exec cp {} "$out/pmc$i.csv" \;
done
cd "$R"
python3 tools/r4/iso_summary.py "$out" > "$out/summary.json" && cat "$out/summary.json"
