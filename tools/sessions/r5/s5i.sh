#!/usr/bin/env bash
# round 5: vectorised fused split-K reducer — bitwise tests, config 2/5 A/B (two rounds)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_drivers.py -k "split_fused or split_reduction or config2 or rows_ks" > gpurun_out/s5i_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/s5i_tests.log; exit 1; }
tail -1 gpurun_out/s5i_tests.log
for r in 1 2; do
for f in 0 1; do
  NERFHIP_SPLIT_FUSED=$f timeout -k 10 200 python3 -u tools/configs_bench.py single wide > gpurun_out/s5i_cfg_f$f.log 2>&1 || { echo "cfg rc=$?"; tail -20 gpurun_out/s5i_cfg_f$f.log; exit 1; }
  echo "fused=$f"; grep '^{' gpurun_out/s5i_cfg_f$f.log | cut -c1-200
done
done
