"""Per-step busy time of every HIP queue in a rocprofv3 kernel trace, and the top kernels of each queue
(steps delimited by the optimizer kernel).  python tools/stream_busy.py TRACE.csv [--last 3] [--top 15]"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--step-kernel", default="(sgd|adam)_kernel")
    ap.add_argument("--full", action="store_true", help="keep template arguments and the grid size in the names")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    idx = [i for i, r in enumerate(rows) if re.search(a.step_kernel, r["Kernel_Name"])]
    steps = list(zip(idx[:-1], idx[1:]))[-a.last:]
    busy = collections.Counter()
    kern = collections.defaultdict(collections.Counter)
    spans = []
    for s0, s1 in steps:
        seg = rows[s0 + 1:s1 + 1]
        spans.append((max(int(r["End_Timestamp"]) for r in seg) - min(int(r["Start_Timestamp"]) for r in seg)) / 1e6)
        for r in seg:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            q = r["Queue_Id"]
            busy[q] += d
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("pg::", "").replace("void ", "")
            n = re.sub(r"\((?!anon).*", "", n)
            kern[q][f"{n} grid={r.get('Grid_Size', r.get('Grid_Size_X', ''))}" if a.full else re.sub(r"<.*", "", n)] += d
    n = len(steps)
    print(f"steps={n} span ms/step={sum(spans) / n:.3f} " + " ".join(f"queue{q}={v / n / 1e3:.3f}ms" for q, v in sorted(busy.items())))
    for q in sorted(kern):
        print(f"-- queue {q}")
        for k, v in kern[q].most_common(a.top):
            print(f"  {v / n:9.1f} us  {k}")


if __name__ == "__main__":
    main()
