#!/usr/bin/env bash
# cos(wz) scratch stores non-temporal (base) vs L2-allocating (v_cost): isolated 40-fit groups + HBM bytes
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3t; mkdir -p $out
BASE=$R/nerf-attention_amd/nerf_attention/_lib/libnerfhip.so
V=$R/build/variants/v_cost.so
for c in medium large; do
  bash $R/tools/ab.sh "--config $c --fits 40 --epochs 41 --precision bf16x3" $BASE $V > $out/ab_$c.log 2>&1 || { tail $out/ab_$c.log; exit 1; }
done
grep -h rep $out/ab_*.log | cut -c1-220
cd /tmp && export TMPDIR=/tmp
for v in base cost; do
  if [ $v = base ]; then L=$BASE; else L=$V; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    NERFHIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $ctr -d $out/${v}_$ctr -o run --output-format csv -- python3 $R/tools/kbench.py --config medium --fits 40 --epochs 10 --repeat 1 --precision bf16x3 > $out/${v}_$ctr.log 2>&1 || { echo "pmc $v $ctr failed"; tail -3 $out/${v}_$ctr.log; exit 1; }
  done
done
python3 - $out <<'PY'
import csv, glob, sys, collections, re
out = sys.argv[1]
for v in ("base", "cost"):
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        acc = collections.defaultdict(list)
        for f in glob.glob(f"{out}/{v}_{ctr}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                m = re.search(r"(k_step_\w+)<([^>]*)>", r["Kernel_Name"])
                if m and r["Counter_Name"] == ctr:
                    acc[m.group(1)].append(float(r["Counter_Value"]))
        print(v, ctr, {k: round(sum(x) / len(x) / 1e3, 1) for k, x in acc.items()}, "MB/launch (KB units)")
PY
