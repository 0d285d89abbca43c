# kernel trace of config 2 (one medium fit) to measure the gaps between the
# epoch's dependent kernels
set -u
R="$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out="$R/gpurun_out/single_trace"; mkdir -p "$out"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/t" -o run --output-format csv -- python3 "$R/tools/configs_bench.py" single > "$out/log" 2>&1 || { echo "trace failed"; tail "$out/log"; exit 1; }
f=$(find "$out/t" -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
step = [r for r in rows if "k_step" in r["Kernel_Name"] or "k_adam" in r["Kernel_Name"]]
# the last 2000 epochs' kernels (the timed fit)
step = step[-6000:]
dur = collections.defaultdict(list); gaps = []
for a, b in zip(step, step[1:]):
    gaps.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
for r in step:
    n = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
    dur[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in dur.items():
    print(f"{n:42s} n={len(v)} mean {sum(v)/len(v):8.2f} us")
gaps.sort()
print(f"gaps between consecutive epoch kernels: median {gaps[len(gaps)//2]:.2f} us, mean {sum(gaps)/len(gaps):.2f} us, p90 {gaps[int(len(gaps)*0.9)]:.2f} us")
t0 = int(step[0]["Start_Timestamp"]); t1 = int(step[-1]["End_Timestamp"])
print(f"span {(t1-t0)/1e6:.2f} ms over {len(step)} kernels")
PY
