#!/usr/bin/env bash
# Round validation: GPU parity suite + smoke, default bench, configs 2 and 5.
set -u
tag="${1:-val}"; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/gputests.log 2>&1 || { tail -30 $out/gputests.log; exit 1; }
tail -2 $out/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
timeout -k 10 300 python -u tools/configs_bench.py single wide > $out/configs.log 2>&1 || { tail $out/configs.log; exit 1; }
grep -v "^W\|amdgpu.ids" $out/configs.log
