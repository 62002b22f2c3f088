"""Host-side profile of one ResNet-50 bs256 training step through the DDP path (run with the 1-rank RCCL
rehearsal environment bench.py uses: PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 MASTER_ADDR/PORT RANK=0
WORLD_SIZE=1).  Prints the host operations longer than --min-us in start order (relative to the step start),
so a stall in the host's issue stream (the GPU then idles) can be attributed to a call.

python tools/ddp_host_profile.py [--min-us 40] [--out gpurun_out/ddp_host.json]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-us", type=float, default=40.0)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from pytorch_distributed_nn_amd.parallel import runtime
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    runtime.init_process_group()
    dev = runtime.device()
    model = build_model("resnet50", num_classes=1000).to(dev)
    net = DistributedDataParallel(model, bucket_cap_mb=32.0)
    opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    x = torch.randn(a.batch, 3, 224, 224, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 1000, (a.batch,), device=dev)
    main_stream = torch.cuda.Stream(device=dev, priority=-1)
    main_stream.wait_stream(torch.cuda.current_stream(dev))

    def step():
        opt.zero_grad()
        with torch.profiler.record_function("fwd"):
            loss = OF.cross_entropy(net(x), y)
        with torch.profiler.record_function("bwd"):
            loss.backward()
        with torch.profiler.record_function("opt"):
            opt.step()

    with torch.cuda.stream(main_stream):
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
            step()
            torch.cuda.synchronize()
    if a.out:
        prof.export_chrome_trace(a.out)
    evs = [e for e in prof.events() if e.time_range.elapsed_us() >= a.min_us]
    t0 = min(e.time_range.start for e in prof.events())
    for e in sorted(evs, key=lambda e: e.time_range.start):
        print(f"{(e.time_range.start - t0) / 1e3:9.3f} ms  {e.time_range.elapsed_us():8.1f} us  thr {e.thread:>6}  {e.name[:90]}")


if __name__ == "__main__":
    main()
