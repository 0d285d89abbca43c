#!/usr/bin/env bash
# (1) the K-split fix (no per-item SGPR operand, no EXEC write near a load):
#     the compile-time forward-only instantiation (the one that failed) and the
#     shipped kernel, two workgroups per CU, 4 repeats each;
# (2) sweep schedule experiments (chunk size, hardware queues), 400 epochs
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/ks_fix_r4c.log; : > $out
V=build/variants
L=nerf-attention_amd/nerf_attention/_lib/libnerfhip.so
for v in $V/v_ksfix2_modes.so $L; do
  echo "## $(basename $v)" >> $out
  KS_CASES="256,2,16384,0;256,2,16384,3;512,2,16384,0;128,1,16384,0;128,1,16384,3" KS_PADS=0 NERFHIP_LIB=$v timeout -k 10 300 python3 tools/r3/ks_probe.py $(basename $v .so) 4 2>&1 | grep -v amdgpu.ids | cut -c1-170 >> $out || { echo "probe rc=$? on $v"; tail -5 $out; exit 1; }
done
grep -c '"bad_blocks": 0,' $out; grep -v '"bad_blocks": 0,' $out | cut -c1-170
out2=gpurun_out/sweep_sched.log; : > $out2
for gm in 40 20 80; do for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q NERFHIP_GROUP_MAX=$gm timeout -k 10 120 python3 tools/r4/sweep_sched.py --epochs 400 --tag "gm$gm-q$q" 2>&1 | grep tag >> $out2 || { echo "sched rc=$?"; exit 1; }
done; done
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 tools/r4/sweep_sched.py --epochs 2000 --steps 1 --tag "default-2000" 2>&1 | grep tag >> $out2 || exit 1
cat $out2
# (3) forced row/param CU mix: dynamic LDS padding (KB) of the regular row /
#     parameter kernels (NERFHIP_ROWS_LDS_PAD / NERFHIP_PARAMS_LDS_PAD)
for pad in "0 0" "8 0" "0 10" "8 2" "6 4"; do set -- $pad
  NERFHIP_ROWS_LDS_PAD=$1 NERFHIP_PARAMS_LDS_PAD=$2 GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python3 tools/r4/sweep_sched.py --epochs 400 --tag "pad-r$1-p$2" 2>&1 | grep tag >> $out2 || { echo "pad rc=$?"; exit 1; }
done
tail -5 $out2
