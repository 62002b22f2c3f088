"""Per-stream occupancy of one training step from a rocprofv3 --kernel-trace CSV (no PMC: real concurrency).

python tools/stream_timeline.py TRACE.csv [--top N]

Takes the last full step of the trace (between the last two optimizer kernels, sgd/adam), then per stream
reports busy time (sum of its kernel intervals: one stream's kernels do not overlap), the gaps between consecutive kernels, and the largest gaps (what the compute stream
waits on); finally the top kernels by time on the critical (compute) stream."""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(({"s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"]), "q": (r["Queue_Id"], r["Stream_Id"]),
                  "n": r["Kernel_Name"]} for r in rows), key=lambda k: k["s"])
    opt = [k for k in ks if "sgd_kernel" in k["n"] or "adam_kernel" in k["n"]]
    if len(opt) < 2:
        print("need >= 2 optimizer kernels")
        return
    # last full step: between the last two optimizer kernels
    t0, t1 = opt[-2]["e"], opt[-1]["e"]
    step = [k for k in ks if k["s"] >= t0 and k["e"] <= t1]
    print(f"step {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
    by = defaultdict(list)
    for k in step:
        by[k["q"]].append(k)
    for q, kk in sorted(by.items(), key=lambda x: -len(x[1])):
        busy, gaps, last = 0, [], None
        for k in kk:
            busy += k["e"] - k["s"]
            if last is not None and k["s"] > last["e"]:
                gaps.append((k["s"] - last["e"], last["n"][:60], k["n"][:60]))
            last = k
        tg = sum(g[0] for g in gaps)
        print(f"queue/stream {q}: {len(kk)} kernels, busy {busy / 1e3:.1f} us, gaps {tg / 1e3:.1f} us "
              f"({len(gaps)}; median {sorted(g[0] for g in gaps)[len(gaps) // 2] / 1e3 if gaps else 0:.1f} us)")
        for g in sorted(gaps, reverse=True)[:5]:
            print(f"   gap {g[0] / 1e3:7.1f} us  after {g[1]}  before {g[2]}")
    main_q = max(by, key=lambda q: len(by[q]))
    # classify the compute stream's gaps: "dep" = the next kernel starts within 4 us of another stream's
    # kernel ending (an event wait on it), "idle" = nothing else was running during the gap (host / launch
    # bound), else "overlap" (another stream busy, no visible dependency)
    others = [k for k in step if k["q"] != main_q]
    cls = defaultdict(lambda: [0, 0])
    kk = by[main_q]
    for a_, b_ in zip(kk, kk[1:]):
        g = b_["s"] - a_["e"]
        if g <= 0:
            continue
        if any(0 <= b_["s"] - o["e"] <= 4000 for o in others):
            c = "dep"
        elif not any(o["s"] < b_["s"] and o["e"] > a_["e"] for o in others):
            c = "idle"
        else:
            c = "overlap"
        cls[c][0] += g
        cls[c][1] += 1
    print("compute-stream gaps by cause: " + ", ".join(f"{c} {t / 1e3:.1f} us ({n})" for c, (t, n) in
                                                      sorted(cls.items())))
    agg = defaultdict(lambda: [0, 0])
    for k in by[main_q]:
        agg[k["n"][:100]][0] += k["e"] - k["s"]
        agg[k["n"][:100]][1] += 1
    print(f"top kernels on {main_q}:")
    for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:a.top]:
        print(f"  {t / 1e3:8.1f} us {c:4d}  {n}")


if __name__ == "__main__":
    main()
