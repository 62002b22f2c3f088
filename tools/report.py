"""Run reports (SURVEY.md §2.3 CPP-14 plot helpers, §2.4 TF-09 benchmark driver percentiles).

    python tools/report.py time-loss  outfiles/time_loss_out_*        # loss / error vs wall time and step
    python tools/report.py timeline   outfiles/timeline_out_*         # gradient arrivals per step
    python tools/report.py percentiles metrics.jsonl [--field backward_ms]   # p50/p80/p90/p95/p99
    python tools/report.py cdf outfiles/compute_times_rank*.jsonl      # per-worker compute-time CDF

File formats (written by parallel/ps.py and the native csrc/runtime/mlp_native.cpp roles):
  time_loss_out_<scheme>:  "step time_ms loss error_rate" per evaluation (MPI_code/src/python/plot_time_loss.py:10-34)
  timeline_out_<scheme>:   "time_ms step 1" at a step start, "time_ms step 0 worker layer" (native) or
                           "time_ms step worker" (python PS) per gradient arrival (visualize_timeline.py:7-66)
  metrics JSONL:           Trainer / bench records with *_ms fields (utils.observability.MetricsSink)

Plots are written as PNG when matplotlib is importable, otherwise the series are printed as CSV.
"""
import argparse
import collections
import json
import sys

import numpy as np


def _plot(series, xlabel, ylabel, out):
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:
        for name, (xs, ys) in series.items():
            print(f"# {name}: {xlabel},{ylabel}")
            for x, y in zip(xs, ys):
                print(f"{x},{y}")
        return None
    plt.figure(figsize=(6, 4))
    for name, (xs, ys) in series.items():
        plt.plot(xs, ys, label=name)
    plt.xlabel(xlabel)
    plt.ylabel(ylabel)
    plt.legend(fontsize=7)
    plt.tight_layout()
    plt.savefig(out)
    return out


def time_loss(files, out):
    series_t, series_s = {}, {}
    for f in files:
        rows = np.loadtxt(f, ndmin=2)
        name = f.split("time_loss_out_")[-1]
        series_t[name] = (rows[:, 1] / 1e3, rows[:, 2])
        series_s[name] = (rows[:, 0], rows[:, 2])
        print(f"{name}: {len(rows)} evaluations, final step {int(rows[-1, 0])}, loss {rows[-1, 2]:.4f}, "
              f"error {rows[-1, 3]:.4f}, wall {rows[-1, 1] / 1e3:.1f}s")
    _plot(series_t, "time (s)", "loss", out + "_time_loss.png")
    _plot(series_s, "step", "loss", out + "_step_loss.png")


def timeline(files):
    for f in files:
        per_step = collections.Counter()
        starts = {}
        lines = [ln.split() for ln in open(f) if not ln.startswith("#")]     # "# stale_dropped ..." summary
        native = any(len(p) >= 5 for p in lines)
        for p in lines:
            if len(p) < 3:
                continue
            t, step = float(p[0]), int(p[1])
            if native and len(p) == 3 and p[2] == "1":
                starts[step] = t
            elif len(p) >= 5:            # native: t step 0 worker layer (count layer-0 arrivals)
                if int(p[4]) == 0:
                    per_step[step] += 1
            else:                        # python PS: t step worker
                per_step[step] += 1
        n = len(per_step)
        avg = sum(per_step.values()) / max(n, 1)
        steps = sorted(starts)
        dur = np.diff([starts[s] for s in steps]) if len(steps) > 1 else np.array([0.0])
        print(f"{f}: {n} steps, average gradients received per step {avg:.2f}, "
              f"mean step time {dur.mean():.2f} ms")


def percentiles(path, field):
    vals = []
    for line in open(path):
        try:
            rec = json.loads(line)
        except ValueError:
            continue
        if rec.get(field) is not None:
            vals.append(float(rec[field]))
    if not vals:
        print(f"no '{field}' values in {path}")
        return
    v = np.asarray(vals)
    qs = {q: float(np.percentile(v, q)) for q in (50, 80, 90, 95, 99)}
    print(json.dumps({"field": field, "n": len(v), "mean": float(v.mean()),
                      **{f"p{q}": round(x, 4) for q, x in qs.items()}}))


def compute_cdf(files, out):
    """Per-worker compute-time CDF and pooled percentiles from compute_times_rank<r>.jsonl files (the TF
    benchmark driver's "time-CDF" curves and p80/p90/p95/p99 prints, distributed_TF/tools/benchmark.py:60-111,
    fed by the timeout manager's per-worker records, distributed_TF/src/timeout_manager.py:48-70)."""
    per = collections.defaultdict(list)
    for f in files:
        for line in open(f):
            try:
                r = json.loads(line)
            except ValueError:
                continue
            if r.get("compute_ms") is not None:
                per[int(r.get("rank", -1))].append(float(r["compute_ms"]))
    if not per:
        print("no compute_ms records")
        return None
    series = {}
    for rank, v in sorted(per.items()):
        v = np.sort(np.asarray(v))
        series[f"rank {rank}"] = (v.tolist(), (np.arange(1, len(v) + 1) / len(v)).tolist())
    pooled = np.concatenate([np.asarray(v) for v in per.values()])
    summary = {"n": int(len(pooled)), "workers": len(per), "mean_ms": float(pooled.mean()),
               **{f"p{q}": round(float(np.percentile(pooled, q)), 4) for q in (50, 80, 90, 95, 99)},
               "slowest_worker": max(per, key=lambda r: float(np.mean(per[r])))}
    print(json.dumps(summary))
    _plot(series, "compute time (ms)", "CDF", f"{out}_compute_cdf.png")
    return summary


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["time-loss", "timeline", "percentiles", "cdf"])
    ap.add_argument("files", nargs="+")
    ap.add_argument("--field", default="backward_ms")
    ap.add_argument("--out", default="report")
    a = ap.parse_args(argv)
    if a.kind == "time-loss":
        time_loss(a.files, a.out)
    elif a.kind == "timeline":
        timeline(a.files)
    elif a.kind == "cdf":
        compute_cdf(a.files, a.out)
    else:
        for f in a.files:
            percentiles(f, a.field)


if __name__ == "__main__":
    sys.exit(main())
