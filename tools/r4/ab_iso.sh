#!/usr/bin/env bash
# A/B library variants on the bench's isolated groups (tools/r4/isokernel.py):
# tools/r4/ab_iso.sh "<isokernel args>" v1.so v2.so ...   (2 interleaved rounds)
args="$1"; shift
for round in 1 2; do
  for v in "$@"; do
    echo "## round $round variant $(basename "$v") args $args"
    NERFHIP_LIB="$v" timeout -k 5 120 python3 tools/r4/isokernel.py $args || exit $?
  done
done
