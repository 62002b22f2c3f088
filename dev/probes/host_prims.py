"""Per-call host cost (us) of the primitives every fused-block launch pays, on the GPU box.

python dev/probes/host_prims.py  -> one JSON line {primitive: us}"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def us(fn, n=20000):
    for _ in range(200):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return round((time.perf_counter() - t0) / n * 1e6, 3)


def main():
    from pytorch_distributed_nn_amd.ops import _backend as B, kernels as K
    dev = torch.device("cuda")
    x = torch.empty(4096, device=dev, dtype=torch.bfloat16)
    s = torch.cuda.Stream(device=dev)
    main_s = torch.cuda.current_stream(dev)
    ev = torch.cuda.Event()
    r = {
        "current_stream(dev)": us(lambda: torch.cuda.current_stream(dev)),
        "current_stream().cuda_stream": us(lambda: torch.cuda.current_stream().cuda_stream),
        "raw_stream": us(lambda: torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())),
        "B.stream()": us(B.stream),
        "torch.empty(cuda)": us(lambda: torch.empty(256, 64, device=dev, dtype=torch.bfloat16)),
        "empty_like": us(lambda: torch.empty_like(x)),
        "view": us(lambda: x.view(64, 64)),
        "data_ptr": us(lambda: x.data_ptr()),
        "record_stream": us(lambda: x.record_stream(s), 5000),
        "event.record": us(lambda: ev.record(s), 5000),
        "wait_event": us(lambda: main_s.wait_event(ev), 5000),
        "K.stream_wait": us(lambda: K.stream_wait(s, main_s), 5000),
        "bn_apply launch": us(lambda: K.bn_apply(x.view(64, 64), torch.ones(64, device=dev),
                                                   torch.zeros(64, device=dev), relu=True), 3000),
        "lib getattr": us(lambda: getattr(B.lib(), "pdnn_stream_wait")),
    }

    def ctx_stream():
        with torch.cuda.stream(s):
            pass
    r["with stream(s)"] = us(ctx_stream, 5000)

    def ctx_dev():
        with torch.cuda.device(dev):
            pass
    r["with device(dev)"] = us(ctx_dev, 5000)
    torch.cuda.synchronize()
    print(json.dumps(r))


if __name__ == "__main__":
    main()
