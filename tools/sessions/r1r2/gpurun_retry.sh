#!/usr/bin/env bash
# Retry a gpurun call ONLY when the box never ran the command (status=transient,
# or exit 3 = no box free).  Any run that started is never repeated.
# usage: tools/gpurun_retry.sh <logfile> <gpurun args...>
log="$1"; shift
for attempt in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    echo "[retry] attempt $attempt: box not available (rc=$rc), waiting" >&2
    sleep 75
    continue
  fi
  exit $rc
done
exit 3
