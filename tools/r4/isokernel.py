"""The bench's isolated leg on its own (development / profiling tool).

Builds the 280-fit sweep exactly as bench.py does, takes the engine's
heaviest group of the dominant width (bench.heaviest_group: the first 40-fit
W = 256 chunk) and runs bench.isolated_kernel on it, so that
`rocprofv3 --kernel-trace --stats -- python3 tools/r4/isokernel.py` profiles
the very launches whose hipEvent average bench.py reports as
roofline.avg_launch_ms.  Prints one JSON line.

usage: python tools/r4/isokernel.py [--width 256] [--epochs 101] [--precision bf16x3]
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES before HIP initialises)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--kernel", default="rows", choices=["rows", "params"])
    ap.add_argument("--epochs", type=int, default=bench.ISO_EPOCHS)
    ap.add_argument("--precision", default="bf16x3", choices=["fp32", "bf16x3"])
    ap.add_argument("--repeat", type=int, default=1)
    args = ap.parse_args()
    from nerf_attention.workloads import sweep_280
    _plan, specs = sweep_280(2048, seed=0)
    sel = bench.heaviest_group(specs, args.width, 0)
    cfgs = [specs[i].config for i in sel]
    fl = (bench.rows_flops if args.kernel == "rows" else bench.params_flops)(2048, 128, cfgs)
    kname = f"k_step_{args.kernel}<{args.width},128>"
    for rep in range(args.repeat):
        r = bench.isolated_kernel([specs[i] for i in sel], kname, fl, args.precision,
                                  bench.PEAK[args.precision], 0, epochs=args.epochs)
        r.update(kernel=kname, precision=args.precision, fits=len(sel), rep=rep,
                 flops_per_launch=fl)
        print(json.dumps(r), flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
