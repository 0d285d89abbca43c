#!/usr/bin/env bash
# Round-3 validation: GPU parity suite + smoke.  usage: tools/r3/validate.sh <tag> [extra pytest args]
set -u
tag="${1:-val}"; shift || true
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $out/gputests.log 2>&1 || { tail -40 $out/gputests.log; exit 1; }
tail -3 $out/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
