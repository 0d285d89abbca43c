#!/usr/bin/env bash
# PMC passes (one rocprofv3 run each, <= 8 SQ counters) over an isolated
# kbench group.  usage: tools/prof_pmc.sh <out_tag> <kbench args...>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
tag="$1"; shift
export TMPDIR=/tmp
out="$R/gpurun_out/pmc_$tag"
mkdir -p "$out"
i=0
for set in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY" \
  "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $set -d "$out/p$i" -o run --output-format csv -- python3 "$R/tools/kbench.py" "$@" --repeat 1) > "$out/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$out/p$i.log"; exit 1; }
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections, re
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)<([^>]*)>", r["Kernel_Name"])
        if not m or not m.group(1).startswith("k_step"): continue
        acc[(m.group(1) + "<" + m.group(2) + ">", r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:40s} {c:28s} {sum(v)/len(v):16.1f}  n={len(v)}")
PY
