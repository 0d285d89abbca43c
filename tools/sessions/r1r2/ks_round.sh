#!/usr/bin/env bash
# K-split: co-residency check, parity subset, timing A/B.
set -u
out=gpurun_out/ks_round_${1:-a}; mkdir -p $out
timeout -k 10 200 python -u tools/ks_diag4.py > $out/diag4.log 2>&1 || { tail $out/diag4.log; exit 1; }
grep -v "^W\|amdgpu.ids" $out/diag4.log
bash tools/ks_ab.sh ${1:-a}
