"""k-of-n straggler mode with no straggler vs the plain DDP path (ResNet-50 bs256, world 1 over a 1-rank RCCL
group): what each part of the k-of-n machinery costs per step.

python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 dev/probes/kofn_tax.py
(PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 in the environment)"""
import contextlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from pytorch_distributed_nn_amd.parallel import runtime
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.optim import SGD
    from pytorch_distributed_nn_amd.optim import flat as FL
    from pytorch_distributed_nn_amd.ops import functional as OF
    runtime.init_process_group()
    dev = runtime.device()
    torch.manual_seed(0)
    xs = [torch.randn(256, 3, 224, 224, device=dev).to(torch.bfloat16) for _ in range(2)]
    ys = [torch.randint(0, 1000, (256,), device=dev) for _ in range(2)]
    res = {}
    variants = [("ddp", dict()), ("kofn", dict(num_aggregate=1)),
                ("kofn_no_throttle", dict(num_aggregate=1, throttle=False)), ("kofn_no_mode", dict(num_aggregate=1)),
                ("ddp_again", dict())]
    ms = torch.cuda.Stream(device=dev, priority=-1)
    ms.wait_stream(torch.cuda.current_stream(dev))
    real_mode = FL.ParamUseMode
    import pytorch_distributed_nn_amd.parallel.ddp as D
    for name, kw in variants:
        D.ParamUseMode = (lambda armed: contextlib.nullcontext()) if name == "kofn_no_mode" else real_mode
        model = build_model("resnet50").to(dev)
        net = DistributedDataParallel(model, **kw)
        opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)

        def step(i):
            opt.zero_grad()
            loss = OF.cross_entropy(net(xs[i % 2]), ys[i % 2])
            if net.kofn is not None:
                net.backward(loss)
            else:
                loss.backward()
            opt.step()
        with torch.cuda.stream(ms):
            for i in range(6):
                step(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(20):
                step(i)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 20
        res[name] = {"ms_per_step": round(dt * 1e3, 3), "img_s": round(256 / dt, 1),
                     "aborted": net.aborted_steps}
        net.close()
        del net, model, opt
        torch.cuda.empty_cache()
        print(json.dumps({name: res[name]}), flush=True)
    D.ParamUseMode = real_mode
    print(json.dumps(res))
    runtime.destroy()


if __name__ == "__main__":
    main()
