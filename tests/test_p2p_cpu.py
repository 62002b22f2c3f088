"""Point-to-point gradient send test (reference comm_test/comm_test.py:38-69,
120-222): rank 1 trains LeNet for one batch and isends each parameter gradient with tag = parameter
index; rank 0 irecvs into buffers of the known shapes.  Here over torch.distributed (gloo on CPU; the same
calls run on RCCL for GPU tensors), with the gradients checked bit-exactly against rank 0's own copy."""
import torch

from dist_utils import run_world


def _p2p(rank, world):
    import torch.distributed as dist
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    torch.manual_seed(0)
    model = build_model("LeNet", 10)
    x = torch.randn(16, 1, 28, 28)
    y = torch.randint(0, 10, (16,))
    params = list(model.parameters())
    if rank == 1:
        OF.cross_entropy(model(x), y).backward()
        reqs = [dist.isend(p.grad.contiguous(), dst=0, tag=i) for i, p in enumerate(params)]
        for r in reqs:
            r.wait()
        return len(reqs)
    bufs = [torch.empty_like(p) for p in params]
    reqs = [dist.irecv(b, src=1, tag=i) for i, b in enumerate(bufs)]
    for r in reqs:
        r.wait()
    OF.cross_entropy(model(x), y).backward()
    return [torch.equal(b, p.grad) for b, p in zip(bufs, params)], [tuple(b.shape) for b in bufs]


def test_p2p_gradient_send():
    res = run_world(_p2p, 2, ())
    ok, shapes = res[0]
    assert all(ok) and len(shapes) == 8 and res[1] == 8              # LeNet: 8 parameter tensors
