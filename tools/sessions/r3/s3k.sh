#!/usr/bin/env bash
# small-tile split-K rule: full GPU suite, configs 2 and 5
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3k; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gputests.log 2>&1 || { tail -40 $out/gputests.log; exit 1; }
tail -2 $out/gputests.log
for i in 1 2; do timeout -k 10 120 python -u tools/configs_bench.py single wide 2>/dev/null | grep ms_per; done | tee $out/configs.log
