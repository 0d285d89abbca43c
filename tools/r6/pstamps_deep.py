"""Workgroup timeline of the parameter kernel on the bench's isolated leg (the
sweep's heaviest W = 256 chunk: 40 deep fits), from a NERFHIP_STAMPS build:

  python tools/build_variant.py pstamps -DNERFHIP_STAMPS --parts 0,6
  NERFHIP_LIB=build/variants/v_pstamps.so python tools/r6/pstamps_deep.py [epochs] [out.json]

Per wave (s_memrealtime, 100 MHz): 0 entry, 1 first loads issued, 2 first block
staged, 3 MFMA loop done, 4 epilogue issued; 5 HW_ID, 6 XCC_ID; 7 the block loop in s_memtime
cycles (high 32 bits) and its barrier-side wait (low 32 bits: from each block's
last MFMA/split issue through its barrier).  The last
epoch's launch is kept.  Reports the workgroup durations of the heavy (MFMA)
tiles, how many run at once over the launch per XCD, and the tail: the time
after the last heavy workgroup STARTED, when the chip can only drain.
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402,F401  (GPU_MAX_HW_QUEUES before HIP initialises)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    out = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "gpurun_out" / "pstamps_deep.json"
    from nerf_attention import _native, engine
    from nerf_attention.workloads import sweep_280
    if not _native.load().nerfhip_build_flags() & 2:
        sys.exit("not a NERFHIP_STAMPS library (set NERFHIP_LIB)")
    _plan, specs = sweep_280(2048, seed=0)
    sel = bench.heaviest_group(specs, 256, 0)
    job = engine.FitJob([specs[i] for i in sel], epochs, devices=[0])
    # the parameter kernel's [4096][4][8] region, then the row kernel's stamps
    # at kRowStampsOff = 2^20 ([blocks][waves][16]; tools/stamps.py reads them)
    n_waves = sum(8 * ((g.n + 7) // 8) * (g.n_pad // 16) for g in job.groups)
    buf = torch.zeros((1 << 20) + 16 * n_waves, dtype=torch.int64, device="cuda")
    os.environ["NERFHIP_PSTAMPS"] = str(buf.data_ptr())   # read when the launch arguments are made
    job.launch()
    job.wait()
    st = buf[:4096 * 4 * 8].view(-1, 4, 8).cpu().numpy().astype(np.int64)
    used = st[:, 0, 0] > 0
    st = st[used]
    w0 = st[:, 0, :]                       # wave 0 of every workgroup
    heavy = w0[:, 4] > 0
    t0 = w0[:, 0].min()
    start = (w0[:, 0] - t0) / 100.0        # µs
    end_all = (st[:, :, 4].max(axis=1) - t0) / 100.0
    end = np.where(heavy, end_all, start)
    xcc = w0[:, 6] & 0xF
    hw = w0[:, 5]
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    dur = end - start
    hv = np.flatnonzero(heavy)
    launch_end = float(end.max())
    last_start = float(start[hv].max())
    res = {"epochs": epochs, "fits": len(sel), "workgroups": int(used.sum()),
           "heavy": int(heavy.sum()), "launch_us": round(launch_end, 2),
           "last_heavy_start_us": round(last_start, 2),
           "tail_us": round(launch_end - last_start, 2),
           "heavy_dur_us": {q: round(float(np.percentile(dur[hv], p)), 2)
                            for q, p in (("min", 0), ("p10", 10), ("p50", 50), ("p90", 90),
                                         ("max", 100))},
           "phases_mean_us": {name: round(float(((w0[hv, k] - w0[hv, k - 1]) / 100.0).mean()), 2)
                              for k, name in ((1, "issue"), (2, "first_block"), (3, "mfma_loop"),
                                              (4, "epilogue"))}}
    # concurrency of heavy workgroups over time (0.5 µs bins), chip and per XCC
    bins = np.arange(0.0, launch_end + 0.5, 0.5)
    conc = np.zeros(len(bins), dtype=int)
    per_x = {}
    for i in hv:
        m = (bins >= start[i]) & (bins < end[i])
        conc += m
        per_x.setdefault(int(xcc[i]), np.zeros(len(bins), dtype=int))[:] += m
    res["heavy_running_hist"] = {f"{b:.0f}us": int(conc[k]) for k, b in enumerate(bins) if k % 20 == 0}
    res["per_xcc"] = {x: {"heavy": int(((xcc == x) & heavy).sum()),
                          "last_end_us": round(float(end[(xcc == x) & heavy].max()), 2),
                          "last_start_us": round(float(start[(xcc == x) & heavy].max()), 2),
                          "peak_running": int(v.max())}
                      for x, v in sorted(per_x.items())}
    # slot 7 (the block loop, s_memtime cycles): barrier-side wait summed over
    # blocks (low 32 bits) and the whole loop (high 32 bits), every heavy wave
    s7 = st[hv, :, 7].astype(np.uint64)
    bw = (s7 & np.uint64(0xFFFFFFFF)).astype(np.float64)
    lp = (s7 >> np.uint64(32)).astype(np.float64)
    ok = lp > 0
    if ok.any():
        frac = bw[ok] / lp[ok]
        loop_us = ((st[hv, :, 3] - st[hv, :, 2]) / 100.0)[ok]
        res["block_loop"] = {
            "barrier_wait_frac": {q: round(float(np.percentile(frac, p)), 3)
                                  for q, p in (("p10", 10), ("p50", 50), ("p90", 90))},
            "barrier_wait_frac_mean": round(float(frac.mean()), 3),
            "loop_cycles_mean": round(float(lp[ok].mean()), 0),
            "memtime_mhz": round(float((lp[ok] / np.maximum(loop_us, 1e-3)).mean()), 1)}
    res["cus_seen"] =int(len({(int(x), int(s), int(c)) for x, s, c in zip(xcc, se, cu)}))
    # heavy workgroups that started in the first 5 µs vs later, and their durations
    first = hv[start[hv] < 5.0]
    later = hv[start[hv] >= 5.0]
    res["first_wave"] = {"n": int(len(first)), "dur_mean_us": round(float(dur[first].mean()), 2)
                         if len(first) else None}
    res["later"] = {"n": int(len(later)), "dur_mean_us": round(float(dur[later].mean()), 2)
                    if len(later) else None}
    out.parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(out.with_suffix(".npz"), st=st)
    out.write_text(json.dumps(res, indent=1))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
