set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "direct or split or batched" --timeout 200 --timeout-method thread > gpurun_out/direct_tests.log 2>&1 || { tail -30 gpurun_out/direct_tests.log; exit 1; }
tail -2 gpurun_out/direct_tests.log
AB_SWEEP=0 AB_CONFIGS="medium:1 large:1 medium:5 large:5 tiny:5 small:5" bash tools/ab_run.sh direct build/variants/v_sgprdma.so build/variants/v_direct.so > /dev/null
grep -v amdgpu.ids gpurun_out/ab_direct/kbench.log | sed 's/"precision": "bf16x3", //'
