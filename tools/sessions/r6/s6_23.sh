#!/usr/bin/env bash
# round 6: bf16x3 scratch as split planes (row kernels store their split
# operand; the parameter kernel stages by LDS-DMA and reads transposed, no
# split) — bitwise A/B against the round-6 start library first; only if equal,
# the isolated deep W = 256 leg (rows + params) and the GPU suite
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_23; mkdir -p $o
NERFHIP_LIB=build/variants/v_base.so timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/base.npz > $o/ab_base.log 2>&1 || { echo "base ab rc=$?"; tail -5 $o/ab_base.log; exit 1; }
timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/new.npz > $o/ab_new.log 2>&1 || { echo "new ab rc=$?"; tail -8 $o/ab_new.log; exit 1; }
python3 - $o/base.npz $o/new.npz <<'PY' | tee $o/ab_cmp.log
import sys, numpy as np
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
print(f"{len(a.files) - len(bad)}/{len(a.files)} arrays bitwise equal")
for k in bad[:12]:
    x, y = a[k].astype(np.float64), b[k].astype(np.float64)
    print(k, "max|d|", float(np.max(np.abs(x - y))), "max|x|", float(np.max(np.abs(x))), "nan", bool(np.isnan(y).any()))
sys.exit(1 if bad else 0)
PY
rc=$?
rm -f $o/base.npz $o/new.npz
[ $rc -eq 0 ] || exit 1
for k in params rows; do
  timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel $k > $o/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $o/iso.log; exit 1; }
  grep '^{' $o/iso.log | cut -c1-160
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/gputests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error" $o/gputests.log | head -20; tail -30 $o/gputests.log; exit 1; }
tail -1 $o/gputests.log
