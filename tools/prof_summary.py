"""Summarise a rocprofv3 kernel trace: per-kernel time over the last `--window-ms` of the trace (steady state)."""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--window-ms", type=float, default=0, help="0 = whole trace")
ap.add_argument("--steps", type=int, default=1, help="divide totals by this many steps")
ap.add_argument("--top", type=int, default=30)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
end = int(rows[-1]["End_Timestamp"])
if a.window_ms:
    rows = [r for r in rows if int(r["Start_Timestamp"]) > end - a.window_ms * 1e6]
tot, cnt = collections.Counter(), collections.Counter()
for r in rows:
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))[:90]
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot[n] += d
    cnt[n] += 1
busy = sum(tot.values())
span = (end - int(rows[0]["Start_Timestamp"])) / 1e6
print(f"kernels={len(rows)} busy={busy/1e6/a.steps:.2f} ms/step span={span/a.steps:.2f} ms/step")
for n, d in tot.most_common(a.top):
    print(f"{d/1e6/a.steps:8.3f} ms {cnt[n]//a.steps:5d}x  {100*d/busy:5.1f}%  {n}")
