set -u
bash tools/gpu_validate.sh r2b || exit 1
for rep in 1 2; do for p in lpt blocked; do
  timeout -k 10 300 python tools/rank_probe.py --epochs 200 --worlds 2,4,8 --all-ranks --partition $p 2>/dev/null | grep world
done; done
