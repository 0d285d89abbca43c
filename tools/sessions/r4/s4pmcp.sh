#!/usr/bin/env bash
# issue / stall counters of the isolated W=256 parameter-kernel leg (two PMC passes)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out/pmc_issue_par
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d "$R/gpurun_out/pmc_issue_par/p1" -o run --output-format csv -- python3 "$R/tools/r4/isokernel.py" --width 256 --kernel params > "$R/gpurun_out/pmc_issue_par/p1.log" 2>&1 || { echo "pass1 rc=$?"; tail -5 "$R/gpurun_out/pmc_issue_par/p1.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE -d "$R/gpurun_out/pmc_issue_par/p2" -o run --output-format csv -- python3 "$R/tools/r4/isokernel.py" --width 256 --kernel params > "$R/gpurun_out/pmc_issue_par/p2.log" 2>&1 || { echo "pass2 rc=$?"; tail -5 "$R/gpurun_out/pmc_issue_par/p2.log"; exit 1; }
cd "$R"
python3 tools/r4/pmc_issue.py --kernel="k_step_params<256, 128, true, false, false" $(find gpurun_out/pmc_issue_par -name '*counter_collection.csv') > gpurun_out/pmc_issue_par/summary.json && cat gpurun_out/pmc_issue_par/summary.json
