#!/usr/bin/env bash
# W=256 row kernel with 8 waves (128-row workgroups, n_pad granule 128) vs 4 waves
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3h; mkdir -p $out
NERFHIP_LIB=build/variants/v_w8.so timeout -k 10 200 python -u tools/bitwise_ab.py /tmp/ab_w8.npz > $out/ab_w8.log 2>&1 || { tail $out/ab_w8.log; exit 1; }
timeout -k 10 200 python -u tools/bitwise_ab.py /tmp/ab_w4.npz > $out/ab_w4.log 2>&1 || { tail $out/ab_w4.log; exit 1; }
python -u tools/bitwise_ab.py --cmp /tmp/ab_w8.npz /tmp/ab_w4.npz | tee $out/ab_cmp.log
python3 - <<'PY' | tee -a $out/ab_cmp.log
import numpy as np
a, b = np.load("/tmp/ab_w8.npz"), np.load("/tmp/ab_w4.npz")
bad = sorted({k.rsplit("_", 2)[0] for k in a.files if not np.array_equal(a[k], b[k])})
print("groups differing:", bad)
PY
for rep in 1 2; do
  for v in w8 base; do
    if [ $v = w8 ]; then export NERFHIP_LIB=build/variants/v_w8.so; else unset NERFHIP_LIB; fi
    timeout -k 10 120 python -u tools/kbench.py --config medium --fits 40 --epochs 41 --repeat 2 --precision bf16x3 2>/dev/null | tail -1 | sed "s/^/$v /" | tee -a $out/kbench.log
  done
done
for v in w8 base w8 base; do
  if [ $v = w8 ]; then export NERFHIP_LIB=build/variants/v_w8.so; else unset NERFHIP_LIB; fi
  timeout -k 10 300 python -u bench.py --epochs 200 --no-cpu-baseline --no-also-fp32 --no-e2e > $out/bench200_$v.log 2>&1 || { tail $out/bench200_$v.log; exit 1; }
  grep '^{"metric' $out/bench200_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" | tee -a $out/bench200.log
done
