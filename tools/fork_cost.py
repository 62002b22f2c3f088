"""Cost of a cross-stream fork on the compute stream (the two-stream ResNet schedule forks ~70 times a step).

python tools/fork_cost.py [--n 400]

A chain of n tiny kernels on a high-priority stream; after each, the low-priority side stream is made to
wait on it and runs a tiny kernel of its own.  Reports the compute stream's time per link for each fork
mechanism: none, torch Stream.wait_stream, the fence-free event (streams.hip pdnn_stream_wait), and a
write-value / wait-value pair (pdnn_stream_wait_value); with and without the side kernel.  Also checks that
the side kernel saw the compute stream's result (ordering)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import _backend  # noqa: E402
from pytorch_distributed_nn_amd.ops._backend import call  # noqa: E402


def fork(mode, side, main):
    if mode == "torch":
        side.wait_stream(main)
    elif mode == "light":
        call("pdnn_stream_wait", side.cuda_stream, main.cuda_stream)
    elif mode == "value":
        call("pdnn_stream_wait_value", side.cuda_stream, main.cuda_stream)


def run(mode, side_work, n, main, side, x, y, chk):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(main):
        e0.record(main)
        for i in range(n):
            x.add_(1.0)
            if mode != "none":
                fork(mode, side, main)
                if side_work:
                    with torch.cuda.stream(side):
                        chk[i] = x[0]            # must read >= base + i + 1
                        y.add_(1.0)
        e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=400)
    a = ap.parse_args()
    assert _backend.available()
    dev = torch.device("cuda")
    main_s = torch.cuda.Stream(device=dev, priority=-1)
    side = torch.cuda.Stream(device=dev, priority=0)
    x = torch.zeros(1 << 20, device=dev)
    y = torch.zeros(1 << 20, device=dev)
    chk = torch.zeros(a.n, device=dev)
    for mode in ("none", "torch", "light", "value"):
        for side_work in ((False,) if mode == "none" else (False, True)):
            try:
                run(mode, side_work, 20, main_s, side, x, y, chk[:20])       # warm-up
            except _backend.HipError as e:
                print(json.dumps({"mode": mode, "error": str(e)}), flush=True)
                break
            base = float(x[0])
            us = run(mode, side_work, a.n, main_s, side, x, y, chk)
            ok = None
            if side_work:
                want = base + torch.arange(1, a.n + 1, device=dev, dtype=torch.float32)
                ok = bool((chk >= want).all())
            print(json.dumps({"mode": mode, "side_kernel": side_work, "us_per_link": round(us, 2),
                              "ordered": ok}), flush=True)


if __name__ == "__main__":
    main()
