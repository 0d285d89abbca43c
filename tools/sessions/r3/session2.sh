#!/usr/bin/env bash
# (1) K-split co-residency bisection: compile-time forward-only kernel (control) and four variants
# (2) parameter-kernel staging permutation: bitwise A/B, isolated timing, LDS bank-conflict counters
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s2; mkdir -p $out
export KS_CASES="256,2,16384,0;256,2,8192,3" KS_PADS=0
for v in ksmodes ksA ksB ksC ksD; do
  NERFHIP_LIB=build/variants/v_$v.so timeout -k 10 200 python -u tools/r3/ks_probe.py $v 3 > $out/ks_$v.jsonl 2> $out/ks_$v.err || { echo "$v failed"; tail -3 $out/ks_$v.err; exit 1; }
  python3 -c "
import json,sys
for l in open('$out/ks_$v.jsonl'):
    r=json.loads(l); print(r['tag'],r['N'],r['E'],r['rep'],'bad_blocks',r['bad_blocks'],'max_err %.2e'%r['max_err'])"
done
unset KS_CASES KS_PADS
timeout -k 10 200 python -u tools/bitwise_ab.py $out/ab_perm.npz > $out/ab_perm.log 2>&1 || { tail $out/ab_perm.log; exit 1; }
NERFHIP_LIB=build/variants/v_pbase.so timeout -k 10 200 python -u tools/bitwise_ab.py $out/ab_base.npz > $out/ab_base.log 2>&1 || { tail $out/ab_base.log; exit 1; }
python -u tools/bitwise_ab.py --cmp $out/ab_perm.npz $out/ab_base.npz | tee $out/ab_cmp.log
for rep in 1 2; do
  for lib in base perm; do
    if [ $lib = base ]; then export NERFHIP_LIB=build/variants/v_pbase.so; else unset NERFHIP_LIB; fi
    for cfg in medium large; do
      timeout -k 10 120 python -u tools/kbench.py --config $cfg --fits 40 --epochs 41 --repeat 2 --precision bf16x3 2>/dev/null | tail -1 | sed "s/^/$lib /" | tee -a $out/kbench_params.log
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in base perm; do
  if [ $lib = base ]; then export NERFHIP_LIB=$R/build/variants/v_pbase.so; else unset NERFHIP_LIB; fi
  for cfg in medium large; do
    timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d $out/pmc_${lib}_$cfg -o run --output-format csv -- python3 $R/tools/kbench.py --config $cfg --fits 40 --epochs 10 --repeat 1 --precision bf16x3 > $out/pmc_${lib}_$cfg.log 2>&1 || { echo "pmc $lib $cfg failed"; tail -3 $out/pmc_${lib}_$cfg.log; exit 1; }
  done
done
python3 - $out <<'PY'
import csv, glob, sys, re, collections, json
res = {}
for d in sorted(glob.glob(sys.argv[1] + "/pmc_*_*/")):
    tag = d.rstrip("/").split("/")[-1]
    acc = collections.defaultdict(list)
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_step_\w+)<([^>]*)>", r["Kernel_Name"])
            if m: acc[(m.group(1) + "<" + m.group(2) + ">", r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in acc.items():
        res.setdefault(tag, {}).setdefault(k, {})[c] = sum(v) / len(v)
for tag, ks in res.items():
    for k, c in ks.items():
        if "params" in k and "SQ_LDS_IDX_ACTIVE" in c:
            print(tag, k, "conflict/active = %.4f" % (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]), c)
json.dump(res, open(sys.argv[1] + "/pmc_params_conflicts.json", "w"), indent=1)
PY
