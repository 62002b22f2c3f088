"""Summarise a rocprofv3 kernel trace: per-kernel time over the last `--window-ms` of the trace (steady state).

``--by-grid`` splits each kernel by its launch grid, so one GEMM kernel template is reported per problem
shape (which tile count / occupancy each call site gets)."""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--window-ms", type=float, default=0, help="0 = whole trace")
ap.add_argument("--steps", type=int, default=1,
                help="summarise the last N full training steps (split at the optimizer kernel) and divide by N")
ap.add_argument("--top", type=int, default=30)
ap.add_argument("--by-grid", action="store_true")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
end = int(rows[-1]["End_Timestamp"])
t0 = None
if a.window_ms:
    rows = [r for r in rows if int(r["Start_Timestamp"]) > end - a.window_ms * 1e6]
else:
    # the last `steps` full steps: between the optimizer kernel that ends step -steps-1 and the last one (the whole
    # trace also holds warm-up and timed steps: dividing all of it by `steps` overstated busy / span)
    opt = [r for r in rows if "sgd_kernel" in r["Kernel_Name"] or "adam_kernel" in r["Kernel_Name"]]
    if len(opt) > a.steps:
        t0, t1 = int(opt[-a.steps - 1]["End_Timestamp"]), int(opt[-1]["End_Timestamp"])
        rows = [r for r in rows if int(r["Start_Timestamp"]) >= t0 and int(r["End_Timestamp"]) <= t1]
        end = t1
tot, cnt = collections.Counter(), collections.Counter()
for r in rows:
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))[:90]
    if a.by_grid:
        g = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        w = r.get("Workgroup_Size_X", "?")
        n = f"{n} grid={g} wg={w}"
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot[n] += d
    cnt[n] += 1
busy = sum(tot.values())
span = (end - (t0 if t0 is not None else int(rows[0]["Start_Timestamp"]))) / 1e6
print(f"kernels={len(rows)} busy={busy/1e6/a.steps:.2f} ms/step span={span/a.steps:.2f} ms/step")
for n, d in tot.most_common(a.top):
    c = cnt[n] / a.steps
    print(f"{d/1e6/a.steps:8.3f} ms {c:6.1f}x {1e3*d/1e6/max(cnt[n],1):8.1f} us/call {100*d/busy:5.1f}%  {n}")
