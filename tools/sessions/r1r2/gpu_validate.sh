#!/usr/bin/env bash
# GPU parity suite + smoke (+ optional round profile): tools/gpu_validate.sh <tag> [profile]
set -u
tag="$1"; out=gpurun_out/val_$tag; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/gputests.log 2>&1; rc=$?
tail -3 $out/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
if [ "${2:-}" = "profile" ]; then
  bash tools/profile_round.sh $tag bf16x3 || exit 1
  cat gpurun_out/prof_$tag/pmc_traffic.json
fi
