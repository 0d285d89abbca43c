"""The bench's e2e leg alone (fit_kv_cache wall clock on the reference's
on-disk format), repeated: python tools/r4/e2e_probe.py [reps]"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for r in range(reps):
    out = bench.e2e_fit_kv_cache(2048, 2000, "bf16x3")
    out.update(rep=r, stream=os.environ.get("NERFHIP_STREAM", "1"),
               cap512=os.environ.get("NERFHIP_GROUP_MAX_512"))
    print(json.dumps(out), flush=True)
