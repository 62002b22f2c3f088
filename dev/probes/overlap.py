"""Which other-stream kernels overlap a given kernel in a rocprofv3 kernel trace (per call, last steps).

usage: python dev/probes/overlap.py trace.csv attn_bwd_dq [--steps 3] [--step-kernel adam_kernel]
Prints, per matching dispatch, its duration and the overlapping kernels of the other queues (overlap in us),
then totals of overlap time by overlapping kernel name."""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("pattern")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--step-kernel", default="adam_kernel")
    ap.add_argument("--per-call", action="store_true")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.step_kernel in r["Kernel_Name"]]
    lo = ends[-a.steps - 1] + 1 if len(ends) > a.steps else 0
    rows = rows[lo:ends[-1] + 1]
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows]
    tot = defaultdict(float)
    n, dur = 0, 0.0
    for s, e, q, k in ev:
        if a.pattern not in k:
            continue
        n += 1
        dur += (e - s) / 1e3
        ov = []
        for s2, e2, q2, k2 in ev:
            if q2 == q or e2 <= s or s2 >= e:
                continue
            o = (min(e, e2) - max(s, s2)) / 1e3
            ov.append((o, k2[:70]))
            tot[k2[:70]] += o
        if a.per_call:
            print(f"{(e - s) / 1e3:7.1f} us  " + "; ".join(f"{k2} {o:.1f}" for o, k2 in ov))
    print(f"{n} calls of {a.pattern}: {dur / a.steps:.1f} us/step")
    for k, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {v / a.steps:8.1f} us/step overlapped by {k}")


if __name__ == "__main__":
    main()
