#!/usr/bin/env bash
# K-split row kernel: parity subset + single-fit / small-group timing A/B.
set -u
out=gpurun_out/ks_${1:-a}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "bf16x3 or ks or forward_plan or custom_op or chunks" > $out/tests.log 2>&1; rc=$?
tail -15 $out/tests.log
[ $rc -eq 0 ] || exit $rc
for ks in 0 1; do
  echo "NERFHIP_ROWS_KS=$ks" >> $out/kbench.log
  NERFHIP_ROWS_KS=$ks timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config medium --fits 1 --epochs 100 >> $out/kbench.log 2>&1 || exit 1
  NERFHIP_ROWS_KS=$ks timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config large --fits 5 --epochs 100 >> $out/kbench.log 2>&1 || exit 1
  NERFHIP_ROWS_KS=$ks timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config medium --fits 8 --epochs 100 >> $out/kbench.log 2>&1 || exit 1
  NERFHIP_ROWS_KS=$ks timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config wide --fits 1 --epochs 30 --seq-len 8192 >> $out/kbench.log 2>&1 || exit 1
done
grep -v "^W\|amdgpu.ids" $out/kbench.log
echo "split 16" >> $out/kbench.log
NERFHIP_GRAD_SPLIT_MAX=16 timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config medium --fits 1 --epochs 100 >> $out/kbench.log 2>&1 || exit 1
NERFHIP_GRAD_SPLIT_MAX=16 timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config large --fits 5 --epochs 100 >> $out/kbench.log 2>&1 || exit 1
NERFHIP_GRAD_SPLIT_MAX=16 timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config wide --fits 1 --epochs 30 --seq-len 8192 >> $out/kbench.log 2>&1 || exit 1
grep -v "^W\|amdgpu.ids" $out/kbench.log | tail -8
