"""Host lead over the GPU per kernel of one training step, from a rocprofv3 --kernel-trace --hip-runtime-trace
run: for every kernel on the compute stream, (GPU start) - (end of the host launch call that enqueued it).
A small lead at a gap means the GPU waited for the host (launch-bound); a large one means the gap is
GPU-side (dispatch, dependencies).

python tools/host_lead.py PREFIX   (PREFIX_kernel_trace.csv and PREFIX_hip_api_trace.csv)"""
import csv
import sys
from collections import defaultdict


def main():
    pre = sys.argv[1]
    ks = list(csv.DictReader(open(pre + "_kernel_trace.csv")))
    api = {r["Correlation_Id"]: r for r in csv.DictReader(open(pre + "_hip_api_trace.csv"))}
    rows = []
    for k in ks:
        a = api.get(k["Correlation_Id"])
        rows.append({"s": int(k["Start_Timestamp"]), "e": int(k["End_Timestamp"]), "n": k["Kernel_Name"],
                     "q": (k["Queue_Id"], k["Stream_Id"]), "h": int(a["End_Timestamp"]) if a else None})
    rows.sort(key=lambda r: r["s"])
    opt = [r for r in rows if "sgd_kernel" in r["n"]]
    t0, t1 = opt[-2]["e"], opt[-1]["e"]
    step = [r for r in rows if t0 <= r["s"] and r["e"] <= t1]
    by = defaultdict(list)
    for r in step:
        by[r["q"]].append(r)
    main_q = max(by, key=lambda q: len(by[q]))
    kk = by[main_q]
    leads = [r["s"] - r["h"] for r in kk if r["h"] is not None]
    leads.sort()
    print(f"compute-stream kernels {len(kk)}; host lead us: min {leads[0] / 1e3:.1f}, p10 {leads[len(leads) // 10] / 1e3:.1f}, "
          f"median {leads[len(leads) // 2] / 1e3:.1f}, max {leads[-1] / 1e3:.1f}")
    print("gaps > 8 us (position, gap, host lead of the next kernel, kernels):")
    for a_, b_ in zip(kk, kk[1:]):
        g = b_["s"] - a_["e"]
        if g > 8000 and b_["h"] is not None:
            print(f"  {(a_['e'] - t0) / 1e3:8.0f} us  gap {g / 1e3:6.1f}  lead {(b_['s'] - b_['h']) / 1e3:8.1f}  "
                  f"{a_['n'][:40]} -> {b_['n'][:40]}")


if __name__ == "__main__":
    main()
