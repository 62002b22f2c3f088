"""Config-sweep driver (TF-09, distributed_TF/tools/benchmark.py:13-292): launch one run per YAML config,
run it to ``--max-steps``, collect its output directory, and report per config the final evaluator loss,
the wall time, steps/s and the compute-time percentiles (p50/p80/p90/p95/p99), plus the time-loss curves.

    python tools/sweep.py configs/sweeps/r*_of_50.yaml --max-steps 2000 --out sweeps/   # 52 procs each
    python tools/sweep.py cfg1.yaml cfg2.yaml --nproc 3 --max-steps 20 --extra "--no-cuda --synthetic"

Runs are local torchrun launches by default; ``--launcher`` takes a command template with {nproc}, {port}
and {args} (e.g. ``python -m pytorch_distributed_nn_amd.cluster run hosts ...`` for a multi-node sweep).
"""
import argparse
import glob
import json
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

DEFAULT_LAUNCHER = (f"{sys.executable} -m torch.distributed.run --nnodes 1 --nproc-per-node {{nproc}} "
                    "--master-addr 127.0.0.1 --master-port {port} -m pytorch_distributed_nn_amd.cli {args}")


def nproc_for(cfg, default):
    """Processes a PS config needs: its ps-workers + the master (+ the evaluator); else ``default``."""
    import yaml
    with open(cfg) as f:
        c = yaml.safe_load(f) or {}
    if c.get("ps-workers"):
        return int(c["ps-workers"]) + 1 + (1 if c.get("evaluator") else 0)
    return default


def run_one(cfg, out, nproc, max_steps, extra, launcher, port, timeout):
    os.makedirs(out, exist_ok=True)
    nproc = nproc_for(cfg, nproc)
    args = f"--config {shlex.quote(cfg)} --max-steps {max_steps} --out-dir {shlex.quote(out)} --compute-times {extra}"
    cmd = launcher.format(nproc=nproc, port=port, args=args)
    t0 = time.time()
    r = subprocess.run(cmd, shell=True, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    wall = time.time() - t0
    open(os.path.join(out, "run.log"), "w").write(r.stdout + "\n" + r.stderr)
    rec = {"config": os.path.basename(cfg), "nproc": nproc, "returncode": r.returncode, "wall_s": round(wall, 2),
           "steps_per_s": round(max_steps / wall, 3) if r.returncode == 0 else None}
    tl = glob.glob(os.path.join(out, "time_loss_out_*"))
    if tl:
        rows = [ln.split() for ln in open(tl[0]) if ln.strip()]
        if rows:
            rec["final_loss"] = float(rows[-1][2])
            rec["final_err"] = float(rows[-1][3])
    ct = glob.glob(os.path.join(out, "compute_times_rank*.jsonl"))
    if ct:
        from report import compute_cdf
        s = compute_cdf(ct, os.path.join(out, "report"))
        if s:
            rec.update({k: s[k] for k in ("p50", "p80", "p90", "p95", "p99")})
    return rec


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--nproc", type=int, default=3)
    ap.add_argument("--max-steps", type=int, default=100)
    ap.add_argument("--out", default="sweeps")
    ap.add_argument("--extra", default="", help="extra cli flags for every run")
    ap.add_argument("--launcher", default=DEFAULT_LAUNCHER)
    ap.add_argument("--port", type=int, default=29651)
    ap.add_argument("--timeout", type=float, default=3600)
    a = ap.parse_args(argv)
    results = []
    for i, cfg in enumerate(a.configs):
        out = os.path.join(a.out, os.path.splitext(os.path.basename(cfg))[0])
        rec = run_one(cfg, out, a.nproc, a.max_steps, a.extra, a.launcher, a.port + i, a.timeout)
        print(json.dumps(rec), flush=True)
        results.append(rec)
    with open(os.path.join(a.out, "summary.jsonl"), "w") as f:
        for r in results:
            f.write(json.dumps(r) + "\n")
    tls = glob.glob(os.path.join(a.out, "*", "time_loss_out_*"))
    if tls:
        from report import time_loss
        time_loss(tls, os.path.join(a.out, "sweep"))
    return results


if __name__ == "__main__":
    main()
