#!/usr/bin/env bash
# round 6: issue / stall counters of the parameter kernel on the isolated deep
# W = 256 chunk (two PMC passes, tools/r4/pmc_issue.py): VALU per MFMA, MFMA
# busy, waits, LDS activity
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; export TMPDIR=/tmp
d="$R/gpurun_out/pmc_params_r6"; mkdir -p "$d"
k="k_step_params<256, 128, true, false, 0, false"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d "$d/p1" -o run --output-format csv -- python3 "$R/tools/r4/isokernel.py" --width 256 --kernel params > "$d/p1.log" 2>&1 || { echo "pass1 rc=$?"; tail -5 "$d/p1.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE -d "$d/p2" -o run --output-format csv -- python3 "$R/tools/r4/isokernel.py" --width 256 --kernel params > "$d/p2.log" 2>&1 || { echo "pass2 rc=$?"; tail -5 "$d/p2.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d "$d/p3" -o run --output-format csv -- python3 "$R/tools/r4/isokernel.py" --width 256 --kernel params > "$d/p3.log" 2>&1 || { echo "pass3 rc=$?"; tail -5 "$d/p3.log"; }
cd "$R"
python3 tools/r4/pmc_issue.py "--kernel=$k" $(find "$d" -name '*counter_collection.csv') > "$d/summary.json" && cat "$d/summary.json"
