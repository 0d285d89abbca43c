#!/usr/bin/env bash
# Group-chunk cap probe: predicted per-rank times (rank_probe) at worlds 1,4,8
# for several NERFHIP_GROUP_MAX values.  usage: bash tools/chunk_probe.sh 40 16 8
for cap in "$@"; do
  echo "## GROUP_MAX=$cap"
  NERFHIP_GROUP_MAX=$cap timeout -k 5 200 python tools/rank_probe.py --epochs 400 --worlds 1,4,8 2>/dev/null || exit $?
done
