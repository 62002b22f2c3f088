"""Host enqueue time vs GPU time per phase (forward / backward / optimizer) of one training step started on an
idle GPU: if the GPU reaches the end of a phase about when the host finishes enqueuing it, the next phase starts
launch-bound.  ResNet-50 bs 256 or GPT-2 small bs 8, plain step, high-priority compute stream like bench.py.

python dev/probes/host_phase.py [--model resnet50|gpt2_small]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    a = ap.parse_args()
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD, AdamW, flatten_module
    dev = torch.device("cuda")
    lm = a.model.startswith("gpt2")
    model = (build_model(a.model) if lm else build_model(a.model, num_classes=1000)).to(dev)
    flatten_module(model)
    if lm:
        opt = AdamW(model.parameters(), lr=6e-4, weight_decay=0.1)
        t = torch.randint(0, 50257, (8, 1025), device=dev)
        x, y = t[:, :-1].contiguous(), t[:, 1:].contiguous()
        fwd = lambda: model(x, y)  # noqa: E731
    else:
        opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
        x = torch.randn(256, 3, 224, 224, device=dev).to(torch.bfloat16)
        y = torch.randint(0, 1000, (256,), device=dev)
        fwd = lambda: OF.cross_entropy(model(x), y)  # noqa: E731
    ms = torch.cuda.Stream(device=dev, priority=-1)
    ms.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(ms):
        for _ in range(5):
            opt.zero_grad()
            fwd().backward()
            opt.step()
        for _ in range(3):
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            h = [time.perf_counter()]
            ev[0].record()
            opt.zero_grad()
            loss = fwd()
            h.append(time.perf_counter())
            ev[1].record()
            loss.backward()
            h.append(time.perf_counter())
            ev[2].record()
            opt.step()
            h.append(time.perf_counter())
            ev[3].record()
            torch.cuda.synchronize()
            hd = [round((h[i] - h[0]) * 1e3, 2) for i in (1, 2, 3)]
            gd = [round(ev[0].elapsed_time(ev[i]), 2) for i in (1, 2, 3)]
            print(f"{a.model}: host enqueue done at fwd {hd[0]} / bwd {hd[1]} / opt {hd[2]} ms;"
                  f"  GPU done at fwd {gd[0]} / bwd {gd[1]} / opt {gd[2]} ms", flush=True)


if __name__ == "__main__":
    main()
