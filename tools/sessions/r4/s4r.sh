#!/usr/bin/env bash
# config 2's per-epoch gap vs the K-split LDS pad (full CU / 80 KB / none)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for pad in full 80 0; do
  d="$R/gpurun_out/cfg2pad_$pad"; mkdir -p "$d"
  env_pad=""; [ "$pad" != full ] && env_pad="NERFHIP_KS_PAD_KB=$pad"
  (cd /tmp && env $env_pad timeout -k 10 180 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 "$R/tools/kbench.py" --config medium --fits 1 --epochs 400 --precision bf16x3 --repeat 1) > "$d.log" 2>&1 || { echo "trace rc=$?"; tail "$d.log"; exit 1; }
  f=$(find "$d" -name '*kernel_trace.csv' | head -1)
  echo "## pad $pad"; python3 tools/r4/gaps.py "$f" | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({'epoch_kernel_us': d['epoch_kernel_us'], 'epoch_gap_us': d['epoch_gap_us'], 'rows_us': d['kernels']['k_step_rows_ks']['median_us']}))"
done
