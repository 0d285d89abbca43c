#!/usr/bin/env bash
set -u
out=gpurun_out/${1:-sp16}; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/gputests.log 2>&1 || { tail -30 $out/gputests.log; exit 1; }
tail -2 $out/gputests.log
timeout -k 10 300 python -u tools/configs_bench.py single wide > $out/configs.log 2>&1 || { tail $out/configs.log; exit 1; }
grep -v "^W\|amdgpu.ids" $out/configs.log
for c in "small --fits 5" "tiny --fits 5" "medium --fits 1"; do
  timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config $c --epochs 100 >> $out/kbench.log 2>&1 || exit 1
done
grep -v "^W\|amdgpu.ids" $out/kbench.log
timeout -k 10 300 python -u tools/rank_probe.py --worlds 8 --all-ranks --partition auto > $out/rank_probe.log 2>&1 || { tail $out/rank_probe.log; exit 1; }
grep -v "^W\|amdgpu.ids" $out/rank_probe.log
