# A/B library variants on the 200-epoch 280-fit sweep (bench.py, untimed kernels).
# usage: bash tools/sweep_ab.sh <reps> lib1.so lib2.so ...
reps=$1; shift
for rep in $(seq 1 $reps); do for lib in "$@"; do
  echo -n "$(basename $lib) rep=$rep "
  NERFHIP_LIB=$lib timeout -k 5 120 python bench.py --epochs 200 --no-cpu-baseline --no-also-fp32 --no-kernel-timing 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
done; done
