"""Checkpoint-polling evaluator (TF-06: distributed_TF/src/nn_eval.py:49-140, entry mnist_eval.py:30-39).

Runs beside a training job: every ``--eval-interval-secs`` it looks for checkpoints in
``--checkpoint-dir`` it has not evaluated yet (the reference restores the newest one per poll,
``tf.train.get_checkpoint_state``), loads each with ``torch.load(weights_only=True)``, evaluates loss /
precision@1 / precision@5 on the test set and appends one JSON record per checkpoint to
``--eval-out`` (the reference writes TF summaries).  It stops after a checkpoint reaching
``--max-steps``, after ``--run-once``, or when no new checkpoint appeared for ``--idle-timeout-secs``.

    python -m pytorch_distributed_nn_amd.evaluator --checkpoint-dir ck --network LeNet --dataset MNIST \\
        --eval-interval-secs 10 --eval-out eval.jsonl
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import time

import torch


def list_checkpoints(ckdir):
    """Complete checkpoint files, oldest first (a checkpoint is written to .tmp and renamed)."""
    fs = [f for f in glob.glob(os.path.join(ckdir, "*.pt")) if not f.endswith(".tmp")]
    return sorted(fs, key=lambda f: (os.path.getmtime(f), f))


def evaluate_checkpoint(path, model, batches, device):
    from .ops import functional as OF
    from .utils.observability import accuracy
    ck = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(ck["state_dict"])
    model.eval()
    tot, p1, p5, n = 0.0, 0.0, 0.0, 0
    with torch.no_grad():
        for x, y in batches:
            x, y = x.to(device), y.to(device)
            out = model(x)
            tot += float(OF.cross_entropy(out, y)) * len(y)
            a1, a5 = accuracy(out.float(), y, (1, min(5, out.shape[1])))
            p1 += float(a1) * len(y)
            p5 += float(a5) * len(y)
            n += len(y)
    return {"checkpoint": os.path.basename(path), "step": int(ck.get("step", 0)), "epoch": int(ck.get("epoch", 0)),
            "loss": tot / max(n, 1), "prec1": p1 / max(n, 1), "prec5": p5 / max(n, 1), "time": time.time()}


def poll(ckdir, model, batches_fn, device, out_path=None, interval_s=10.0, max_steps=None, idle_timeout_s=600.0,
         run_once=False, printer=print):
    """Evaluate every new checkpoint in ``ckdir`` as it appears; returns the records."""
    done, recs = set(), []
    last_new = time.time()
    while True:
        new = [f for f in list_checkpoints(ckdir) if f not in done]
        for f in new:
            rec = evaluate_checkpoint(f, model, batches_fn(), device)
            done.add(f)
            recs.append(rec)
            last_new = time.time()
            printer(f"Eval {rec['checkpoint']} step {rec['step']}: loss {rec['loss']:.4f} "
                    f"prec@1 {rec['prec1']:.2f} prec@5 {rec['prec5']:.2f}")
            if out_path:
                with open(out_path, "a") as fo:
                    fo.write(json.dumps(rec) + "\n")
        if run_once or (max_steps and any(r["step"] >= max_steps for r in recs)):
            return recs
        if time.time() - last_new > idle_timeout_s:
            return recs
        time.sleep(interval_s)


def main(argv=None):
    from .cli import add_fit_args
    from .data.datasets import DataLoader, dataset_from_args
    from .models import build_model
    ap = add_fit_args(argparse.ArgumentParser(description="checkpoint-polling evaluator"))
    ap.add_argument("--eval-interval-secs", type=float, default=10.0)
    ap.add_argument("--idle-timeout-secs", type=float, default=600.0)
    ap.add_argument("--eval-batches", type=int, default=10)
    ap.add_argument("--eval-out", type=str, default=None)
    ap.add_argument("--run-once", action="store_true")
    a = ap.parse_args(argv)
    dev = torch.device("cpu") if a.no_cuda or not torch.cuda.is_available() else torch.device("cuda")
    _, test_ds = dataset_from_args(a.dataset, a.data_dir, a.synthetic, dev, a.test_batch_size, a.network)
    nc = 1000 if a.dataset.upper() == "IMAGENET" else 10
    model = build_model(a.network, nc).to(dev)
    bs = min(a.test_batch_size, len(test_ds))

    def batches():
        dl = DataLoader(test_ds, bs, "cpu")
        try:
            for _ in range(a.eval_batches):
                x, y = dl.next_batch()
                yield x.float(), y
        finally:
            dl.close()

    return poll(a.checkpoint_dir, model, batches, dev, a.eval_out, a.eval_interval_secs, a.max_steps,
                a.idle_timeout_secs, a.run_once)


if __name__ == "__main__":
    main()
