"""Per-(kernel, grid) roofline of a rocprofv3 PMC run (layout of tools/pmc_summary.py: q1/q2/q3 counter CSVs).

python tools/pmc_dispatch.py DIR [--steps N] [--top T] [--hbm-tbs 5.0]

Groups dispatches by kernel name + grid + workgroup size (one group ~ one layer shape), and reports per call:
time, bf16 MFMA TFLOP/s, HBM bytes (FETCH_SIZE doubled + WRITE_SIZE), achieved TB/s, and the roofline floor
max(flops / 2.5 PF, bytes / HBM) with the slack (time - floor) per step -- the ranking of what is worth
optimising.  Dispatches of the three passes are matched by their order (same program, same sequence)."""
import argparse
import csv
import os
from collections import defaultdict

PEAK = 2.5e15


def rows(path):
    out = {}
    if not os.path.exists(path):
        return out
    with open(path) as f:
        for r in csv.DictReader(f):
            d = out.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": r["Grid_Size"],
                                                       "wg": r["Workgroup_Size"], "t": 0})
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                d["t"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--hbm-tbs", type=float, default=5.0)
    a = ap.parse_args()
    q1 = rows(os.path.join(a.dir, "q1_counters.csv"))
    q2 = rows(os.path.join(a.dir, "q2_counters.csv"))
    q3 = rows(os.path.join(a.dir, "q3_counters.csv"))
    g = defaultdict(lambda: defaultdict(float))
    for i, d in enumerate(q1):
        key = (d["name"], d["grid"], d["wg"])
        k = g[key]
        k["n"] += 1
        k["t"] += d["t"]
        k["fl"] += 512 * d.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0)
        if i < len(q2) and q2[i]["name"] == d["name"]:
            k["rd"] += 2 * 1024 * q2[i].get("FETCH_SIZE", 0.0)
        if i < len(q3) and q3[i]["name"] == d["name"]:
            k["wr"] += 1024 * q3[i].get("WRITE_SIZE", 0.0)
    hbm = a.hbm_tbs * 1e12
    tab = []
    for (name, grid, wg), k in g.items():
        n = k["n"]
        t = k["t"] / n * 1e-9
        fl, by = k["fl"] / n, (k["rd"] + k["wr"]) / n
        floor = max(fl / PEAK, by / hbm)
        tab.append((k["n"] / a.steps * (t - floor), name, grid, wg, k["n"] / a.steps, t, fl, by, floor))
    tab.sort(key=lambda r: -r[0])
    tot_t = sum(r[4] * r[5] for r in tab)
    tot_floor = sum(r[4] * r[8] for r in tab)
    print(f"kernel time {tot_t * 1e3:.2f} ms/step, roofline floor {tot_floor * 1e3:.2f} ms/step "
          f"(HBM {a.hbm_tbs} TB/s, bf16 {PEAK / 1e15} PF)")
    print(f"{'slack ms':>8} {'calls':>5} {'us/call':>8} {'floor us':>8} {'TF/s':>6} {'GB':>6} {'TB/s':>5}  kernel [grid/wg]")
    for slack, name, grid, wg, calls, t, fl, by, floor in tab[:a.top]:
        short = name.replace("(anonymous namespace)::", "").split("(")[0][:60]
        print(f"{slack * 1e3:8.3f} {calls:5.1f} {t * 1e6:8.1f} {floor * 1e6:8.1f} {fl / t / 1e12:6.0f} "
              f"{by / 1e9:6.3f} {by / t / 1e12:5.2f}  {short} [{int(grid) // int(wg)}x{wg}]")


if __name__ == "__main__":
    main()
