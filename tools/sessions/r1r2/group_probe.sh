# Sweep throughput vs group splitting (NERFHIP_GROUP_MAX) and HW queue count.
# usage: bash tools/group_probe.sh "<queues list>" "<cap list>" [reps]
for rep in $(seq 1 ${3:-1}); do
for q in $1; do
  for cap in $2; do
    printf "queues=%s group_max=%s rep=%s  " $q $cap $rep >&2
    GPU_MAX_HW_QUEUES=$q NERFHIP_GROUP_MAX=$cap timeout -k 5 120 python bench.py --epochs 200 --no-cpu-baseline --no-also-fp32 --no-kernel-timing | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
  done
done
done
