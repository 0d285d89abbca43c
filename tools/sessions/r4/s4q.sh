#!/usr/bin/env bash
# config 2 (one medium fit, seq 2048): kernel trace -> per-epoch launch gaps
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out/cfg2trace
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace -d "$R/gpurun_out/cfg2trace" -o run --output-format csv -- python3 "$R/tools/kbench.py" --config medium --fits 1 --epochs 400 --precision bf16x3 --repeat 1) > gpurun_out/cfg2trace.log 2>&1 || { echo "trace rc=$?"; tail gpurun_out/cfg2trace.log; exit 1; }
f=$(find gpurun_out/cfg2trace -name '*kernel_trace.csv' | head -1)
python3 tools/r4/gaps.py "$f" | tee gpurun_out/cfg2_gaps.json
