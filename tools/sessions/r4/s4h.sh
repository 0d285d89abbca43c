#!/usr/bin/env bash
# K-split fix check: the compile-time forward-only instantiation (the one that
# failed) built from the fixed source, two workgroups per CU; the shipped
# kernel likewise; config-2 timing of the fix against the pre-fix build.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/ks_fix_r4.log; : > $out
V=build/variants
L=nerf-attention_amd/nerf_attention/_lib/libnerfhip.so
for v in $V/v_ksfix_modes.so $L; do
  echo "## $(basename $v)" >> $out
  KS_CASES="256,2,16384,0;256,2,16384,3;512,2,16384,0;128,1,16384,0;256,2,8192,0" KS_PADS=0 NERFHIP_LIB=$v timeout -k 10 300 python3 tools/r3/ks_probe.py $(basename $v .so) 3 2>&1 | grep -v amdgpu.ids | cut -c1-200 >> $out || { echo "probe rc=$? on $v"; tail -5 $out; exit 1; }
done
echo "## config 2 (one medium fit, seq 2048), K-split rows: pre-fix vs fixed" >> $out
for round in 1 2; do for v in $V/v_base.so $L; do
  echo "# $(basename $v)" >> $out
  NERFHIP_LIB=$v timeout -k 10 120 python3 tools/kbench.py --config medium --fits 1 --epochs 400 --precision bf16x3 --repeat 1 2>&1 | grep rep >> $out || exit 1
done; done
cat $out
