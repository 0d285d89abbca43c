# Isolated per-group kernel timings for both precisions.
set -e
for p in fp32 bf16x3; do
  python tools/kbench.py --config large --fits 40 --epochs 20 --precision $p --repeat 2 | tail -1
  python tools/kbench.py --config medium,deep,hifreq,lofreq --fits 160 --epochs 20 --precision $p --repeat 2 | tail -1
  python tools/kbench.py --config small --fits 40 --epochs 20 --precision $p --repeat 2 | tail -1
  python tools/kbench.py --config tiny --fits 40 --epochs 20 --precision $p --repeat 2 | tail -1
done
