"""Which HIP stream is current inside an autograd final callback (queue_callback) when backward() is called
under a non-default stream?  The fused ResNet backward queues its end-of-backward side-stream join as such a
callback, so the join must land on the stream the optimizer runs on.

python tools/callback_stream_probe.py"""
import json

import torch


class _Probe(torch.autograd.Function):
    seen = {}

    @staticmethod
    def forward(ctx, x):
        return x * 2

    @staticmethod
    def backward(ctx, g):
        _Probe.seen["node"] = torch.cuda.current_stream(g.device).cuda_stream

        def cb():
            _Probe.seen["callback"] = torch.cuda.current_stream(g.device).cuda_stream
        torch.autograd.Variable._execution_engine.queue_callback(cb)
        return g * 2


def main():
    dev = torch.device("cuda")
    s = torch.cuda.Stream(device=dev, priority=-1)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        x = torch.ones(16, device=dev, requires_grad=True)
        _Probe.apply(x).sum().backward()
    torch.cuda.synchronize()
    out = {"caller": s.cuda_stream, "default": torch.cuda.default_stream(dev).cuda_stream, **_Probe.seen}
    out["callback_on_caller"] = out.get("callback") == s.cuda_stream
    out["node_on_caller"] = out.get("node") == s.cuda_stream
    print(json.dumps(out))


if __name__ == "__main__":
    main()
