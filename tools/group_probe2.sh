for rep in 1 2; do for c in 40 20 16; do
  echo -n "large_cap=$c rep=$rep "
  NERFHIP_GROUP_MAX_512=$c timeout -k 5 120 python bench.py --epochs 200 --no-cpu-baseline --no-also-fp32 --no-kernel-timing 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
done; done
