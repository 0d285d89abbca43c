set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r2a/gputests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r2a/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2a/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/r2a/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r2a/bench.log 2>&1 || { echo bench failed; tail gpurun_out/r2a/bench.log; exit 1; }
tail -c 3000 gpurun_out/r2a/bench.log
