#!/usr/bin/env bash
# last check of the committed tree: GPU suite + smoke
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/r3fc; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gputests.log 2>&1 || { tail -40 $out/gputests.log; exit 1; }
tail -1 $out/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
