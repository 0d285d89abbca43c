#!/usr/bin/env bash
set -u
out=gpurun_out/adam; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/gputests.log 2>&1 || { tail -30 $out/gputests.log; exit 1; }
tail -2 $out/gputests.log
for i in 1 2; do
  timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config medium --fits 1 --epochs 200 >> $out/kbench.log 2>&1 || exit 1
done
grep -v "^W\|amdgpu.ids" $out/kbench.log
timeout -k 10 300 python -u tools/configs_bench.py single > $out/configs.log 2>&1 || { tail $out/configs.log; exit 1; }
grep -v "^W\|amdgpu.ids" $out/configs.log
