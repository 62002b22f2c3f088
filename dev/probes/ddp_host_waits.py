"""Where does the host block in the DDP-path ResNet-50 step?  Wraps torch.distributed.all_reduce / broadcast and
Work.wait with host timers, runs bench.py's step at world 1 (PDNN_FORCE_PG + PDNN_DDP_FORCE_COMM) and prints the
calls that took longer than 100 us on the host, plus per-phase host vs device times."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.getcwd())
os.environ.setdefault("PDNN_FORCE_PG", "1")
os.environ.setdefault("PDNN_DDP_FORCE_COMM", "1")
from pytorch_distributed_nn_amd.parallel import runtime  # noqa: E402

slow = []


def wrap(mod, name):
    f = getattr(mod, name)

    def g(*a, **k):
        t = time.perf_counter()
        r = f(*a, **k)
        dt = time.perf_counter() - t
        if dt > 1e-4:
            slow.append((name, round(dt * 1e6)))
        if r is not None and hasattr(r, "wait"):
            w = r.wait

            def ww(*aa, **kk):
                t2 = time.perf_counter()
                rr = w(*aa, **kk)
                d2 = time.perf_counter() - t2
                if d2 > 1e-4:
                    slow.append((name + ".wait", round(d2 * 1e6)))
                return rr
            try:
                r.wait = ww
            except Exception:
                pass
        return r
    setattr(mod, name, g)


for n in ("all_reduce", "broadcast"):
    wrap(dist, n)

from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel  # noqa: E402
from pytorch_distributed_nn_amd.models import build_model  # noqa: E402
from pytorch_distributed_nn_amd.optim import SGD  # noqa: E402
from pytorch_distributed_nn_amd.ops import functional as OF  # noqa: E402

runtime.init_process_group()
dev = runtime.device()
model = build_model("resnet50").to(dev)
net = DistributedDataParallel(model, bucket_cap_mb=32)
opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
x = torch.randn(256, 3, 224, 224, device=dev).to(torch.bfloat16)
y = torch.randint(0, 1000, (256,), device=dev)
ms = torch.cuda.Stream(device=dev, priority=-1)
ms.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(ms):
    for it in range(12):
        if it == 4:
            slow.clear()
        t0 = time.perf_counter()
        opt.zero_grad()
        t1 = time.perf_counter()
        out = net(x)
        t2 = time.perf_counter()
        loss = OF.cross_entropy(out, y)
        loss.backward()
        t3 = time.perf_counter()
        opt.step()
        t4 = time.perf_counter()
        if it >= 4:
            print(f"step {it}: zero {1e3*(t1-t0):.2f} fwd {1e3*(t2-t1):.2f} bwd {1e3*(t3-t2):.2f} opt {1e3*(t4-t3):.2f} ms (host)",
                  flush=True)
    torch.cuda.synchronize()
print("host calls > 100 us:", slow)
runtime.destroy()
