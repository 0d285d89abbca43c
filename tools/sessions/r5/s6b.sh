#!/usr/bin/env bash
# round 5: issue / stall counters of the isolated heaviest-W=256 row leg, 16-row kernel vs 32-row kernel
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out/pmc_issue_r05
export TMPDIR=/tmp
for v in 0 1; do
  d="$R/gpurun_out/pmc_issue_r05/rows32_$v"; mkdir -p "$d"
  cd /tmp
  NERFHIP_ROWS32=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d "$d/p1" -o run --output-format csv -- python3 "$R/tools/r4/isokernel.py" --width 256 --kernel rows > "$d/p1.log" 2>&1 || { echo "pass1 v$v rc=$?"; tail -5 "$d/p1.log"; exit 1; }
  NERFHIP_ROWS32=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE -d "$d/p2" -o run --output-format csv -- python3 "$R/tools/r4/isokernel.py" --width 256 --kernel rows > "$d/p2.log" 2>&1 || { echo "pass2 v$v rc=$?"; tail -5 "$d/p2.log"; exit 1; }
  cd "$R"
  k="k_step_rows<256, 128, true, true"; [ "$v" = 1 ] && k="k_step_rows32<256, 128, true"
  python3 tools/r4/pmc_issue.py "--kernel=$k" $(find "$d" -name '*counter_collection.csv') > "$d/summary.json" && echo "== rows32=$v" && cat "$d/summary.json"
done
