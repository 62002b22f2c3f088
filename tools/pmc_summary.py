"""Per-kernel PMC summary of a rocprofv3 `--pmc` run (dev/gpu_runs/r4_08.sh layout).

python tools/pmc_summary.py DIR [--steps N] [--top T]

DIR holds q1_counters.csv (SQ_INSTS_VALU_MFMA_MOPS_BF16, SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES,
SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE, GRBM_GUI_ACTIVE), optionally q2_counters.csv (FETCH_SIZE, KiB)
and q3_counters.csv (WRITE_SIZE, KiB).  Per kernel name it reports dispatch time, bf16 MFMA FLOPs
(512 x MOPS), achieved TFLOP/s and % of the 2.5 PFLOP/s dense bf16 peak, the LDS bank-conflict ratio and
the L2<->fabric bytes.  FETCH_SIZE is reported doubled (MI355X_MICROARCH.md: on gfx950 it counts half the
bytes of a wide coalesced stream), so "rd" is an upper estimate for scattered reads.
"""
import argparse
import csv
import os
from collections import defaultdict

PEAK_BF16 = 2.5e15


def load(path):
    """dispatch id -> {"name", "t_ns", counter: value}"""
    out = {}
    if not os.path.exists(path):
        return out
    with open(path) as f:
        for r in csv.DictReader(f):
            d = out.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"], "t_ns": 0})
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                d["t_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=3, help="training steps in the profiled program")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--ledger", action="store_true", help="also print read / written GB per step by kernel family")
    a = ap.parse_args()
    q1 = load(os.path.join(a.dir, "q1_counters.csv"))
    trace = os.path.join(a.dir, "q1_trace.csv")
    if os.path.exists(trace):  # counter CSVs of some rocprofv3 builds carry no timestamps
        with open(trace) as f:
            for r in csv.DictReader(f):
                d = q1.get(r["Dispatch_Id"])
                if d is not None and not d["t_ns"]:
                    d["t_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    by_name = defaultdict(lambda: defaultdict(float))
    for d in q1.values():
        k = by_name[d["name"]]
        k["n"] += 1
        k["t"] += d["t_ns"]
        for c in ("SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES",
                  "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE"):
            k[c] += d.get(c, 0.0)
    for fn, cn, key in (("q2_counters.csv", "FETCH_SIZE", "rd"), ("q3_counters.csv", "WRITE_SIZE", "wr")):
        for d in load(os.path.join(a.dir, fn)).values():
            by_name[d["name"]][key] += d.get(cn, 0.0) * 1024 * (2 if key == "rd" else 1)
    tot_t = sum(k["t"] for k in by_name.values())
    tot_fl = sum(512 * k["SQ_INSTS_VALU_MFMA_MOPS_BF16"] for k in by_name.values())
    mm_t = sum(k["t"] for k in by_name.values() if k["SQ_INSTS_VALU_MFMA_MOPS_BF16"] > 0)
    print(f"dispatches={sum(int(k['n']) for k in by_name.values())} kernel-time={tot_t / 1e6 / a.steps:.2f} ms/step "
          f"(PMC-serialised) bf16 MFMA work={tot_fl / 1e12 / a.steps:.3f} TFLOP/step")
    print(f"whole step: {tot_fl / max(tot_t, 1) / 1e3:.0f} TFLOP/s over all kernel time; "
          f"MFMA kernels: {tot_fl / max(mm_t, 1) / 1e3:.0f} TFLOP/s over {mm_t / max(tot_t, 1) * 100:.0f}% of the time")
    print(f"{'ms/step':>8} {'calls':>6} {'TFLOP/s':>8} {'%peak':>6} {'ldsconf':>7} {'rd GB/s':>8} {'wr GB/s':>8}  kernel")
    rows = sorted(by_name.items(), key=lambda kv: -kv[1]["t"])[:a.top]
    for name, k in rows:
        t = max(k["t"], 1.0)
        fl = 512 * k["SQ_INSTS_VALU_MFMA_MOPS_BF16"]
        conf = k["SQ_LDS_BANK_CONFLICT"] / k["SQ_LDS_IDX_ACTIVE"] if k["SQ_LDS_IDX_ACTIVE"] else 0.0
        print(f"{k['t'] / 1e6 / a.steps:8.3f} {k['n'] / a.steps:6.1f} {fl / t / 1e3:8.1f} "
              f"{100 * fl / t * 1e9 / PEAK_BF16:6.1f} {conf:7.3f} {k['rd'] / t:8.0f} {k['wr'] / t:8.0f}  {name[:90]}")
    if a.ledger:
        fam = defaultdict(lambda: defaultdict(float))
        for name, k in by_name.items():
            f = family(name, k)
            for c in ("t", "rd", "wr"):
                fam[f][c] += k[c]
        print(f"\nbyte ledger per step (rd = 2 x FETCH_SIZE: an upper estimate; wr = WRITE_SIZE)")
        print(f"{'family':28} {'ms':>7} {'rd GB':>7} {'wr GB':>7} {'GB/s':>6}")
        tot = defaultdict(float)
        for f, k in sorted(fam.items(), key=lambda kv: -(kv[1]["rd"] + kv[1]["wr"])):
            for c in ("t", "rd", "wr"):
                tot[c] += k[c]
            print(f"{f:28} {k['t'] / 1e6 / a.steps:7.3f} {k['rd'] / 1e9 / a.steps:7.2f} {k['wr'] / 1e9 / a.steps:7.2f} "
                  f"{(k['rd'] + k['wr']) / max(k['t'], 1):6.0f}")
        print(f"{'total':28} {tot['t'] / 1e6 / a.steps:7.3f} {tot['rd'] / 1e9 / a.steps:7.2f} {tot['wr'] / 1e9 / a.steps:7.2f} "
              f"{(tot['rd'] + tot['wr']) / max(tot['t'], 1):6.0f}")


FAMILIES = (("bn_bwd_apply", "BN backward apply"), ("bn_bwd_reduce", "BN backward reduce"),
            ("bn_apply", "BN apply (fwd)"), ("bn_slab_fused", "BN finalize"), ("bn_stats", "BN statistics"),
            ("maxpool_bwd_bnred", "stem pool/BN"), ("bn_relu_maxpool", "stem pool/BN"),
            ("slab_reduce", "split-K / slab reduces"), ("sgd", "optimizer"), ("adam", "optimizer"),
            ("xent", "loss"), ("copyBuffer", "copies / fills"), ("fill", "copies / fills"),
            ("avgpool", "pooling"), ("maxpool", "pooling"))


def family(name, k):
    for key, f in FAMILIES:
        if key in name:
            return f
    if k["SQ_INSTS_VALU_MFMA_MOPS_BF16"] > 0 or any(s in name for s in ("gemm", "conv", "stem")):
        return "MFMA GEMM / conv"
    return "other"


if __name__ == "__main__":
    main()
