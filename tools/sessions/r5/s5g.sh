#!/usr/bin/env bash
# round 5: fused split-K Adam (bitwise tests + config 2/5 A/B), interleaved rows32 timing
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/r5/split_fused_probe.py > gpurun_out/split_fused_probe2.log 2>&1 || { echo "probe rc=$?"; tail -30 gpurun_out/split_fused_probe2.log; exit 1; }
grep "^{" gpurun_out/split_fused_probe2.log | cut -c1-420
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_parity.py -k "split_fused or split_reduction" > gpurun_out/s5g_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/s5g_tests.log; exit 1; }
tail -3 gpurun_out/s5g_tests.log
for f in 0 1; do
  NERFHIP_SPLIT_FUSED=$f timeout -k 10 200 python3 -u tools/configs_bench.py single wide > gpurun_out/s5g_cfg_f$f.log 2>&1 || { echo "cfg rc=$?"; tail -20 gpurun_out/s5g_cfg_f$f.log; exit 1; }
  echo "fused=$f"; grep '^{' gpurun_out/s5g_cfg_f$f.log
done
timeout -k 10 240 python3 -u tools/r5/rows32_check.py > gpurun_out/rows32_check3.log 2>&1 || { echo "check rc=$?"; tail -30 gpurun_out/rows32_check3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rows32_check3.log
