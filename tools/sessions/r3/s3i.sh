#!/usr/bin/env bash
# 8-wave W=256 row kernel: size of the result differences vs the 4-wave kernel (bitwise_ab arrays)
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3i; mkdir -p $out
NERFHIP_LIB=build/variants/v_w8.so timeout -k 10 200 python -u tools/bitwise_ab.py /tmp/ab_w8.npz > $out/ab_w8.log 2>&1 || { tail $out/ab_w8.log; exit 1; }
timeout -k 10 200 python -u tools/bitwise_ab.py /tmp/ab_w4.npz > $out/ab_w4.log 2>&1 || { tail $out/ab_w4.log; exit 1; }
NERFHIP_LIB=build/variants/v_w8.so timeout -k 10 200 python -u tools/bitwise_ab.py /tmp/ab_w8b.npz > $out/ab_w8b.log 2>&1 || { tail $out/ab_w8b.log; exit 1; }
python3 - <<'PY' | tee $out/diff.log
import numpy as np
a, b, a2 = np.load("/tmp/ab_w8.npz"), np.load("/tmp/ab_w4.npz"), np.load("/tmp/ab_w8b.npz")
print("w8 run-to-run bitwise:", all(np.array_equal(a[k], a2[k]) for k in a.files))
for k in a.files:
    if not np.array_equal(a[k], b[k]):
        d = np.abs(a[k].astype(np.float64) - b[k])
        print(k, "max|d| %.3e" % d.max(), "n_diff", int((d > 0).sum()), "of", d.size, "max|x| %.3e" % np.abs(b[k]).max())
PY
