#!/usr/bin/env bash
# Run named GPU steps in order on the gpurun box; each step has its own time
# limit.  A crash-class exit (timeout 124/137, abort 134, segfault 139, or a
# negative Python signal code) stops the script: nothing else touches the GPU.
# An ordinary failure (e.g. pytest assertion, rc 1) is logged and the next step
# runs.  Usage: tools/gpu_steps.sh "name|seconds|command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
status=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"
  secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/${name}.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/${name}.log"
  case $rc in
    0) ;;
    124|137|134|139|250|251|252|253|254|255) echo "=== stop: crash-class exit $rc"; exit $rc ;;
    *) status=$rc ;;
  esac
done
exit $status
