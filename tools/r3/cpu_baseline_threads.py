"""The bench's CPU baseline leg at several torch thread counts on this host
(round 3: repeat spread vs CFS throttling under the GPU box's CPU quota).
usage: python tools/r3/cpu_baseline_threads.py 16 12"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

base = bench.host_cpus
for n in [int(a) for a in sys.argv[1:]]:
    bench.host_cpus = lambda n=n: dict(base(), threads=n)
    r = bench.cpu_baseline(2048, 100)
    print(json.dumps({"threads": n, "value": round(r["value"], 4), "repeat_spread": r["repeat_spread"],
                      "spread_per_arch": r["spread_per_arch"],
                      "throttled_s": r["host"].get("throttled_s_during_baseline"),
                      "per_epoch_ms": r["per_epoch_ms"]}), flush=True)
