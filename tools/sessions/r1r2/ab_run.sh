#!/usr/bin/env bash
# A/B of library variants: isolated groups (kbench) + the 200-epoch sweep.
# usage: tools/ab_run.sh <tag> <variant.so> ...
set -u
tag="$1"; shift
out=gpurun_out/ab_$tag; mkdir -p $out
CONFIGS="${AB_CONFIGS:-medium:40 large:40 medium:1 large:1 small:40 tiny:40}"
for cc in $CONFIGS; do
  c="${cc%%:*} --fits ${cc##*:}"
  echo "## $c" >> $out/kbench.log
  bash tools/ab.sh "--config $c --epochs 20 --precision bf16x3" "$@" >> $out/kbench.log 2>&1 || { echo "kbench failed: $c"; tail -3 $out/kbench.log; exit 1; }
done
[ "${AB_SWEEP:-1}" = "1" ] && for round in 1 2; do
  for v in "$@"; do
    NERFHIP_LIB="$v" timeout -k 10 200 python bench.py --epochs 200 --no-cpu-baseline --no-also-fp32 --no-e2e --no-kernel-timing > $out/sweep_$(basename $v)_$round.json 2>/dev/null || { echo "sweep failed $v"; exit 1; }
    echo "sweep $round $(basename $v) $(python -c "import json,sys; d=json.loads(open('$out/sweep_$(basename $v)_$round.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" >> $out/kbench.log
  done
done
cat $out/kbench.log
