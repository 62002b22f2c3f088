"""Parameter-server mode on CPU/gloo (PAR-DP-PS / PAR-DP-KILL / PAR-DP-BACKUP; SURVEY.md §5.3 fault
injection: sleep-based stragglers as in pure_py_code/distributed_worker.py:131-132)."""
import os
import tempfile

import pytest
import torch

from dist_utils import run_world


def _data(seed=0, n=512):
    g = torch.Generator().manual_seed(seed)
    centers = torch.randn(10, 784, generator=g) * 2
    y = torch.randint(0, 10, (n,), generator=g)
    x = centers[y] + 0.5 * torch.randn(n, 784, generator=g)
    return x, y


def _ps_job(rank, world, comm_type, k, straggler, out_dir, steps):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ps import PSConfig, run_ps
    torch.manual_seed(0)
    model = build_model("mlp2", 10)
    x, y = _data()
    cfg = PSConfig(comm_type=comm_type, num_aggregate=k, evaluator=True, eval_interval=5, lr=0.05, momentum=0.5,
                   max_steps=steps, out_dir=out_dir, inject_straggler=straggler)

    def batches():
        i = 0
        while True:
            sl = slice((i * 32) % 512, (i * 32) % 512 + 32)
            yield x[sl], y[sl]
            i += 1

    def evaluate(m):
        with torch.no_grad():
            out = m(x)
            return float(OF.cross_entropy(out, y)), float((out.argmax(1) != y).float().mean())

    res = run_ps(model, cfg, torch.device("cpu"), loss_fn=OF.cross_entropy, batches=batches(), eval_fn=evaluate)
    # every rank ends with identical weights (final push)
    w = torch.cat([p.detach().flatten() for p in model.parameters()])
    return res, w


@pytest.mark.parametrize("comm_type", ["Bcast", "Async"])
def test_ps_full_sync_learns(comm_type):
    out = tempfile.mkdtemp()
    res = run_world(_ps_job, 4, (comm_type, 0, {}, out, 20))
    master_log, evaluator_rows = res[0][0], res[1][0]
    assert all(r["count"] == 2 for r in master_log)                 # both workers every step
    assert evaluator_rows[-1][2] < evaluator_rows[0][2]             # loss decreased
    for r in res[1:]:
        assert torch.equal(r[1], res[0][1])
    assert any(f.startswith("time_loss_out_") for f in os.listdir(out))


def test_ps_k_of_n_kill_with_straggler():
    """k=1 of 2 workers, rank 3 sleeps 30 ms per layer: it is killed (aborts its backward) and the
    master averages over the real count (1)."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_job, 4, ("Bcast", 1, {3: 30}, out, 8))
    master_log = res[0][0]
    aborted_rank3 = res[3][0]
    assert all(r["count"] == 1 for r in master_log)
    assert sum(2 in r["arrived"] for r in master_log) >= 6          # the fast worker wins most steps
    assert aborted_rank3 >= 4                                       # straggler was short-circuited


def _ps_job_cfg(rank, world, cfg_kw, out_dir, steps):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ps import PSConfig, run_ps
    torch.manual_seed(0)
    model = build_model("mlp2", 10)
    x, y = _data()
    cfg = PSConfig(lr=0.05, max_steps=steps, out_dir=out_dir, **cfg_kw)

    def batches():
        i = 0
        while True:
            sl = slice((i * 32) % 512, (i * 32) % 512 + 32)
            yield x[sl], y[sl]
            i += 1

    res = run_ps(model, cfg, torch.device("cpu"), loss_fn=OF.cross_entropy, batches=batches())
    w = torch.cat([p.detach().flatten() for p in model.parameters()])
    return res, w


def test_ps_backup_workers_drop_stragglers():
    """PAR-DP-BACKUP: collect the first 2 of 3 workers' gradients each step; the slow worker's late
    gradients are dropped as stale and it short-circuits its backward."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_job_cfg, 4, ({"n_to_collect": 2, "inject_straggler": {3: 25}}, out, 8))
    master_log = res[0][0]
    assert all(r["count"] == 2 for r in master_log)
    assert sum(3 in r["arrived"] for r in master_log) <= 2          # the straggler rarely makes the cut
    for r in res[1:]:
        assert torch.equal(r[1], res[0][1])                         # consistent final weights


def test_ps_interval_mode_closes_steps_on_timer():
    """PAR-DP-INTERVAL (TF TimeoutReplicasOptimizer): a step closes interval_ms after its first gradient
    with whatever arrived; a worker slower than the interval is left out."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_job_cfg, 3, ({"interval_ms": 5.0, "inject_straggler": {2: 60}}, out, 6))
    master_log = res[0][0]
    assert all(1 <= r["count"] <= 2 for r in master_log)
    assert sum(r["count"] == 1 for r in master_log) >= 4            # the timer closed most steps early


def _ps_stream_job(rank, world, cfg_kw, out_dir, steps):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ps import PSConfig, run_ps
    torch.manual_seed(0)
    model = build_model("mlp_cpp", 10)
    x, y = _data()
    cfg = PSConfig(lr=0.05, max_steps=steps, out_dir=out_dir, bucket_cap_mb=0.5, first_bucket_mb=0.05, **cfg_kw)

    def batches():
        i = 0
        while True:
            sl = slice((i * 32) % 512, (i * 32) % 512 + 32)
            yield x[sl], y[sl]
            i += 1

    res = run_ps(model, cfg, torch.device("cpu"), loss_fn=OF.cross_entropy, batches=batches())
    return res


def test_ps_streams_gradients_per_bucket():
    """Gradients reach the master bucket by bucket as backward produces them (reverse parameter order),
    visible as several arrivals per worker per step in the arrival timeline."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_stream_job, 3, ({"comm_type": "Async"}, out, 4))
    log = res[0]
    nb = len(log[0]["bucket_counts"])
    assert nb >= 3 and all(r["bucket_counts"] == [2] * nb for r in log)
    tl = [line.split() for line in open(os.path.join(out, [f for f in os.listdir(out)
                                                           if f.startswith("timeline_out_")][0]))]
    per = {}
    for t, step, w, b in tl:
        per.setdefault((int(step), int(w)), []).append((float(t), int(b)))
    for key, arr in per.items():
        assert [b for _, b in arr] == list(range(nb)), (key, arr)     # bucket 0 (last layers) first


def test_ps_interval_without_shortcircuit_drops_late_worker():
    """with shortcircuit off and k-of-n off, a worker slower than the interval keeps computing,
    but its gradients arrive after the step closed and must NOT be averaged in."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_stream_job, 4, ({"interval_ms": 60.0, "shortcircuit": False,
                                         "inject_straggler": {3: 15}}, out, 4))
    log = res[0]
    for r in log[1:]:
        assert 3 not in r["arrived"], r                  # the straggler never delivers a full gradient
        assert min(r["bucket_counts"]) < 3, r            # its late buckets (the first layers) were dropped
    assert res[3] == 0                                   # and it was never aborted (short-circuit off)
