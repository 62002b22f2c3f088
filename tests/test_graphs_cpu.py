"""GraphedStep on the CPU: capture is a GPU feature, so CPU tensors take the eager path with identical
results; the fused optimizers refuse graph mode without a flat CUDA arena."""
import copy

import pytest
import torch


def test_graphed_step_cpu_is_eager():
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD, flatten_module
    from pytorch_distributed_nn_amd.utils.graphs import GraphedStep
    torch.manual_seed(0)
    a = build_model("LeNet", 10)
    b = copy.deepcopy(a)
    oa, ob = SGD(a.parameters(), lr=0.05, momentum=0.9), SGD(b.parameters(), lr=0.05, momentum=0.9)
    gs = GraphedStep(b, ob, loss_fn=OF.cross_entropy)
    x, y = torch.randn(8, 1, 28, 28), torch.randint(0, 10, (8,))
    for _ in range(4):
        oa.zero_grad()
        la = OF.cross_entropy(a(x), y)
        la.backward()
        oa.step()
        lb = gs(x, y)
        assert torch.allclose(la, lb)
    assert gs.graph is None and gs.replays == 0
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb)
    with pytest.raises(RuntimeError):
        flatten_module(b)
        ob.graph_mode(True)


def test_trainer_graph_flag_cpu():
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.optim import SGD
    from pytorch_distributed_nn_amd.trainer import Trainer
    m = build_model("mlp2", 10)
    tr = Trainer(m, SGD(m.parameters(), lr=0.1), graph=True, printer=lambda *a: None)
    assert tr.graph_step is None                    # CPU device: eager
