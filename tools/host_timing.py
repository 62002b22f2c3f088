"""Host vs GPU timeline of the ResNet-50 bs256 train step (same setup as bench.py's 1-GPU path).

python tools/host_timing.py [--batch 256] [--steps 10]

For each phase boundary (step start, forward issued, loss issued, backward issued, optimizer issued) prints
the host time since the step started and the GPU time at which that point's CUDA event completes: where
the host time exceeds the GPU time the GPU waits for launches (host-bound), otherwise the host is ahead."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--cpu-profile", action="store_true", help="torch.profiler CPU table of one step")
    a = ap.parse_args()
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.optim import SGD, flatten_module
    from pytorch_distributed_nn_amd.ops import functional as OF
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = build_model(a.model).to(dev)
    flatten_module(model)
    opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    x = torch.randn(a.batch, 3, 224, 224, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 1000, (a.batch,), device=dev)
    ms = torch.cuda.Stream(device=dev, priority=-1)
    ms.wait_stream(torch.cuda.current_stream(dev))
    names = ["start", "fwd", "loss", "bwd", "opt"]
    with torch.cuda.stream(ms):
        rows = []
        for it in range(a.steps + 3):
            ev = [torch.cuda.Event(enable_timing=True) for _ in names]
            th = []
            th.append(time.perf_counter()); ev[0].record()
            opt.zero_grad()
            out = model(x)
            th.append(time.perf_counter()); ev[1].record()
            loss = OF.cross_entropy(out, y)
            th.append(time.perf_counter()); ev[2].record()
            loss.backward()
            th.append(time.perf_counter()); ev[3].record()
            opt.step()
            th.append(time.perf_counter()); ev[4].record()
            rows.append((th, ev))
        torch.cuda.synchronize()
        if a.cpu_profile:
            from torch.profiler import ProfilerActivity, profile
            with profile(activities=[ProfilerActivity.CPU], record_shapes=False) as prof:
                opt.zero_grad()
                loss = OF.cross_entropy(model(x), y)
                t_b = time.perf_counter()
                loss.backward()
                t_e = time.perf_counter()
                opt.step()
            torch.cuda.synchronize()
            print(f"backward host time {1e3 * (t_e - t_b):.2f} ms")
            print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))
    print(f"{'phase':8s} {'host ms':>9s} {'gpu ms':>9s}   (since step start, mean of {a.steps} steps)")
    hs = [0.0] * len(names)
    gs = [0.0] * len(names)
    for th, ev in rows[3:]:
        for k in range(len(names)):
            hs[k] += (th[k] - th[0]) * 1e3 / a.steps
            gs[k] += ev[0].elapsed_time(ev[k]) / a.steps
    for k, n in enumerate(names):
        print(f"{n:8s} {hs[k]:9.2f} {gs[k]:9.2f}")
    steps = [rows[i + 1][1][0] for i in range(3, len(rows) - 1)]
    per = sum(rows[i][1][0].elapsed_time(rows[i + 1][1][0]) for i in range(3, len(rows) - 1)) / (len(rows) - 4)
    hper = sum(rows[i + 1][0][0] - rows[i][0][0] for i in range(3, len(rows) - 1)) / (len(rows) - 4) * 1e3
    print(f"GPU step {per:.2f} ms, host step {hper:.2f} ms")


if __name__ == "__main__":
    main()
