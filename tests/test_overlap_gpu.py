"""Optimizer step overlapped with the backward (optim/overlap.py): AdamW chunks launched on a side stream
from the grad-ready hooks == the fused whole-arena step after the backward, for GPT-2 over three steps
(the update vs a second plain copy gives the fp32-atomics noise floor)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_backward_overlapped_adamw_matches_step():
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.optim import AdamW, flatten_module
    from pytorch_distributed_nn_amd.optim.overlap import BackwardOverlappedStep
    torch.manual_seed(0)
    m0 = build_model("gpt2_tiny")
    ms = [copy.deepcopy(m0).cuda() for _ in range(3)]
    opts = []
    for m in ms:
        flatten_module(m)
        opts.append(AdamW(m.parameters(), lr=1e-3, weight_decay=0.1))
    ov = BackwardOverlappedStep(opts[2], chunk_mb=0.25, first_mb=0.05)
    assert len(ov.chunks) >= 4
    p0 = ms[0]._pdnn_flat.data.clone()
    g = torch.Generator().manual_seed(1)
    for _ in range(3):
        d = torch.randint(0, 512, (2, 65), generator=g).cuda()
        x, y = d[:, :-1].contiguous(), d[:, 1:].contiguous()
        for i, (m, o) in enumerate(zip(ms, opts)):
            o.zero_grad()
            if i == 2:
                ov.arm()
            m(x, y).backward()
            if i != 2:
                o.step()
    torch.cuda.synchronize()
    assert ov.steps == 3
    fa, fb, fc = (m._pdnn_flat for m in ms)
    upd = (fa.data - p0).norm()
    floor = ((fb.data - fa.data).norm() / upd).item()
    err = ((fc.data - fa.data).norm() / upd).item()
    assert err < 3 * floor + 1e-3, (err, floor)
    # bf16 shadow refreshed by the chunk kernels
    assert ((fc.shadow.float() - fc.data).norm() / fc.data.norm()).item() < 5e-3
    ov.close()
