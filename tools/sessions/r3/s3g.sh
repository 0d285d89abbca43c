#!/usr/bin/env bash
# k_step_rows2 (two row halves per wave) vs k_step_rows: bitwise A/B, isolated timing, 200-epoch sweep
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3g; mkdir -p $out
timeout -k 10 200 python -u tools/bitwise_ab.py /tmp/ab_r2.npz > $out/ab_r2.log 2>&1 || { tail $out/ab_r2.log; exit 1; }
NERFHIP_ROWS2=0 timeout -k 10 200 python -u tools/bitwise_ab.py /tmp/ab_r1.npz > $out/ab_r1.log 2>&1 || { tail $out/ab_r1.log; exit 1; }
python -u tools/bitwise_ab.py --cmp /tmp/ab_r2.npz /tmp/ab_r1.npz | tee $out/ab_cmp.log
for rep in 1 2; do
  for v in 1 0; do
    NERFHIP_ROWS2=$v timeout -k 10 120 python -u tools/kbench.py --config medium --fits 40 --epochs 41 --repeat 2 --precision bf16x3 2>/dev/null | tail -1 | sed "s/^/rows2=$v /" | tee -a $out/kbench.log
  done
done
for v in 1 0; do
  NERFHIP_ROWS2=$v timeout -k 10 300 python -u bench.py --epochs 200 --no-cpu-baseline --no-also-fp32 --no-e2e > $out/bench200_$v.log 2>&1 || { tail $out/bench200_$v.log; exit 1; }
  tail -1 $out/bench200_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rows2=$v', d['value'], d['ms_per_step'], d.get('cos_delta_vs_ref'))" | tee -a $out/bench200.log
done
