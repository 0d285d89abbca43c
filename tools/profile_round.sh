#!/usr/bin/env bash
# Round profile of the bench workload: kernel-trace stats + two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs, MI355X_MICROARCH.md §HBM) over a
# 200-epoch sweep.  Outputs under gpurun_out/prof_<tag>/.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
tag="${1:-x3}"; prec="${2:-bf16x3}"
out="$R/gpurun_out/prof_$tag"
mkdir -p "$out"
export TMPDIR=/tmp
B="$R/bench.py --epochs 200 --no-cpu-baseline --no-also-fp32 --no-e2e --precision $prec"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 $B > "$out/trace.log" 2>&1 || { echo "trace rc=$?"; tail "$out/trace.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- python3 $B > "$out/fetch.log" 2>&1 || { echo "fetch rc=$?"; tail "$out/fetch.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- python3 $B > "$out/write.log" 2>&1 || { echo "write rc=$?"; tail "$out/write.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$out/mfma" -o run --output-format csv -- python3 $B > "$out/mfma.log" 2>&1 || { echo "mfma rc=$?"; tail "$out/mfma.log"; exit 1; }
f=$(find "$out/fetch" -name '*counter_collection.csv' | head -1)
w=$(find "$out/write" -name '*counter_collection.csv' | head -1)
m=$(find "$out/mfma" -name '*counter_collection.csv' | head -1)
python3 "$R/tools/pmc_traffic.py" "$f" "$w" "$out/pmc_traffic.json" "$m" > /dev/null
cp "$m" "$out/mfma_counter_collection.csv"
find "$out/trace" -name '*kernel_stats.csv' -exec cp {} "$out/kernel_stats.csv" \;
echo "profile done: $out"
