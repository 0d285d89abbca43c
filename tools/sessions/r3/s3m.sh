#!/usr/bin/env bash
# is the K-split row kernel bound by cold (post-Adam) weight reads? launch it twice per epoch
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3m; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
NERFHIP_LIB=$R/build/variants/v_twice.so timeout -k 10 120 rocprofv3 --kernel-trace -d $out/t -o run --output-format csv -- python3 $R/tools/configs_bench.py single --epochs 200 > $out/t.log 2>&1 || { tail -3 $out/t.log; exit 1; }
python3 - $out <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/t/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
first, second = [], []
for i in range(1, len(seq)):
    if "rows_ks" in seq[i][0] and "rows_ks" in seq[i - 1][0]:
        second.append(seq[i][1]); first.append(seq[i - 1][1])
import statistics as st
print("pairs", len(first), "first (after Adam) us", round(st.median(first), 2), "second (L2-warm) us", round(st.median(second), 2))
PY
rm -rf $out/t
