"""TF-stack parity on CPU: staircase LR decay, per-worker compute-time records + CDF
percentiles, the checkpoint-polling evaluator, sweep configs."""
import glob
import json
import os
import subprocess
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cli(args, env=None, timeout=240):
    e = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29731", **(env or {}))
    return subprocess.run([sys.executable, "-m", "pytorch_distributed_nn_amd.cli", *args], cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


def test_staircase_lr_decay_and_compute_times_and_poll_evaluator(tmp_path):
    ck, out = tmp_path / "ck", tmp_path / "out"
    r = _cli(["--no-cuda", "--synthetic", "--network", "LeNet", "--dataset", "MNIST", "--batch-size", "16",
              "--epochs", "3", "--lr", "0.1", "--lr-decay-factor", "0.5", "--epochs-per-decay", "1",
              "--checkpoint-dir", str(ck), "--out-dir", str(out), "--compute-times", "--metrics",
              str(tmp_path / "m.jsonl"), "--log-interval", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(x) for x in open(out / "compute_times_rank0.jsonl")]
    assert len(recs) == 12 and all(x["compute_ms"] > 0 for x in recs)      # 64 synthetic / 16 = 4 steps x 3
    from tools.report import compute_cdf
    s = compute_cdf([str(out / "compute_times_rank0.jsonl")], str(tmp_path / "rep"))
    assert s["n"] == 12 and s["p50"] <= s["p99"]
    # evaluator polls the checkpoint directory and evaluates each checkpoint once
    from pytorch_distributed_nn_amd import evaluator
    ev = tmp_path / "eval.jsonl"
    recs = evaluator.main(["--no-cuda", "--synthetic", "--network", "LeNet", "--dataset", "MNIST",
                           "--checkpoint-dir", str(ck), "--eval-out", str(ev), "--run-once",
                           "--test-batch-size", "32", "--eval-batches", "2"])
    assert len(recs) == 3 and sorted(r["epoch"] for r in recs) == [1, 2, 3]
    assert len(open(ev).readlines()) == 3


def test_lr_schedule_staircase():
    lr0, f, decay = 0.1, 0.5, 4
    sched = lambda step: lr0 * f ** (step // decay)  # noqa: E731  (the cli's schedule)
    assert [sched(s) for s in (0, 3, 4, 8)] == [0.1, 0.1, 0.05, 0.025]


def test_sweep_configs_mirror_reference_cfgs():
    files = sorted(glob.glob(os.path.join(ROOT, "configs", "sweeps", "*.yaml")))
    cfgs = [yaml.safe_load(open(f)) for f in files]
    rs = sorted(c["n-to-collect"] for c in cfgs if "n-to-collect" in c)
    ivs = sorted(c["interval-ms"] for c in cfgs if "interval-ms" in c)
    assert rs == [1, 10, 20, 30, 40, 49, 50] and ivs == [3000, 4000, 5000, 6000, 7000]
    from pytorch_distributed_nn_amd.cli import parse_args
    for f in files:
        parse_args(["--config", f])                           # every key is a known flag


def test_sweep_driver_runs_configs(tmp_path):
    cfgs = []
    for name, kv in (("r1", "n-to-collect: 1"), ("iv", "interval-ms: 50")):
        p = tmp_path / f"{name}.yaml"
        p.write_text(f"network: mlp2\ndataset: MNIST\nbatch-size: 16\nmode: ps\nevaluator: true\neval-interval: 2\n{kv}\n")
        cfgs.append(str(p))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from sweep import main
    res = main([*cfgs, "--nproc", "4", "--max-steps", "6", "--out", str(tmp_path / "sw"),
                "--extra", "--no-cuda --synthetic", "--port", "29871"])
    assert [r["returncode"] for r in res] == [0, 0], open(tmp_path / "sw" / "r1" / "run.log").read()[-3000:]
    assert all("p90" in r and "final_loss" in r for r in res)
