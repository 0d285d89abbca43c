#!/usr/bin/env bash
# HEAD check after a container re-creation: GPU parity + smoke, default bench,
# single-fit kernel breakdown.  usage: tools/r2_head_check.sh <tag>
set -u
tag="${1:-head}"; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/gputests.log 2>&1 || { tail -30 $out/gputests.log; exit 1; }
tail -2 $out/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-400
timeout -k 10 120 python -u tools/kbench.py --config medium --fits 1 --epochs 50 > $out/kbench_single.log 2>&1 || { tail $out/kbench_single.log; exit 1; }
timeout -k 10 120 python -u tools/kbench.py --config wide --fits 1 --epochs 20 --seq-len 8192 >> $out/kbench_single.log 2>&1 || { tail $out/kbench_single.log; exit 1; }
cat $out/kbench_single.log
