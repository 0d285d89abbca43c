"""Where the e2e leg's wall clock goes: bench.e2e_fit_kv_cache under
cProfile (warm run after one unprofiled run), plus wall-clock marks of the
streaming driver's phases.  python tools/r4/e2e_timeline.py"""
import cProfile
import io
import json
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from nerf_attention import engine, fit  # noqa: E402

marks = []
T0 = [0.0]
orig_launch, orig_finished = engine.StreamingJob._launch, engine.StreamingJob.finished
orig_stream = fit.train_plan_streaming


def _launch(self, gi):
    orig_launch(self, gi)
    marks.append(("launch", gi, len(self.plan[gi][1]), self.plan[gi][0].W
                  if hasattr(self.plan[gi][0], "W") else None, time.perf_counter()))


def finished(self, poll_s=0.002):
    for gi in orig_finished(self, poll_s):
        marks.append(("done", gi, 0, None, time.perf_counter()))
        yield gi


def stream(*a, **k):
    marks.append(("train_plan_streaming_enter", -1, 0, None, time.perf_counter()))
    r = orig_stream(*a, **k)
    marks.append(("train_plan_streaming_exit", -1, 0, None, time.perf_counter()))
    return r


engine.StreamingJob._launch = _launch
engine.StreamingJob.finished = finished
fit.train_plan_streaming = stream

print(json.dumps(bench.e2e_fit_kv_cache(2048, 2000, "bf16x3")), flush=True)
marks.clear()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
out = bench.e2e_fit_kv_cache(2048, 2000, "bf16x3")
pr.disable()
print(json.dumps(out), flush=True)
base = marks[0][4] if marks else t0
for m in marks:
    print(f"{m[0]:<28} g{m[1]:<3} n={m[2]:<3} t={m[4] - base:8.3f}")
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumtime").print_stats(35)
print(s.getvalue())
