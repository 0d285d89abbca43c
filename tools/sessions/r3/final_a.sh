#!/usr/bin/env bash
# round 3: full GPU parity suite + smoke, then the exact default bench command
set -u
R="$GRAFT_REPO_ROOT"; tag="${1:-r3a}"; out=$R/gpurun_out/$tag; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gputests.log 2>&1 || { tail -40 $out/gputests.log; exit 1; }
tail -2 $out/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1 || { tail $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-400
