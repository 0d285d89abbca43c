set -u
for v in "$@"; do
  echo "== $v"
  NERFHIP_LIB=$v timeout -k 10 300 python tools/rank_probe.py --epochs 200 --worlds 8 --all-ranks --partition lpt 2>/dev/null | grep world
done
