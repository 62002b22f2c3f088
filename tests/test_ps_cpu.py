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


def _ps_job_port_taken(rank, world, out_dir, steps):
    """Every rank holds a listening socket on MASTER_PORT + 1 (and + 2) for the whole job: the port the control
    plane used to take blind.  The job must still run."""
    import socket
    held = []
    for off in (1, 2):
        s = socket.socket()
        try:
            s.bind(("0.0.0.0", int(os.environ["MASTER_PORT"]) + off))
            s.listen(1)
            held.append(s)
        except OSError:       # another rank (or process) holds it already: occupied either way
            s.close()
    try:
        return _ps_job_cfg(rank, world, {"comm_type": "Async"}, out_dir, steps)
    finally:
        for s in held:
            s.close()


def test_ps_control_plane_survives_occupied_master_port_plus_one():
    """the PS store binds an ephemeral port and publishes it over the process group, so a busy
    MASTER_PORT + 1 cannot stop the job."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_job_port_taken, 3, (out, 4))
    assert len(res[0][0]) == 4 and all(r["count"] == 2 for r in res[0][0])
    assert torch.equal(res[1][1], res[0][1]) and torch.equal(res[2][1], res[0][1])


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


# ---------------------------------------------------------------------------------------------- round 3
def _ps_opt_job(rank, world, cfg_kw, out_dir, steps):
    """Workers take different batches (rank-dependent), so the master's averaged gradient is a real mean."""
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ps import PSConfig, run_ps
    torch.manual_seed(0)
    model = build_model("mlp2", 10)
    x, y = _data()
    cfg = PSConfig(max_steps=steps, out_dir=out_dir, **cfg_kw)

    def batches():
        i = 0
        while True:
            j = 2 * i + (rank - 1)
            yield x[j * 32:(j + 1) * 32], y[j * 32:(j + 1) * 32]
            i += 1

    res = run_ps(model, cfg, torch.device("cpu"), loss_fn=OF.cross_entropy, batches=batches())
    w = torch.cat([p.detach().flatten() for p in model.parameters()])
    return res, w


def _reference_run(opt_name, steps, lr, decay=(1.0, 0)):
    """Single process: the same model, the mean of the two workers' gradients, torch's optimizer."""
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    torch.manual_seed(0)
    model = build_model("mlp2", 10)
    x, y = _data()
    opt = {"adam": lambda ps: torch.optim.Adam(ps, lr=lr), "adamw": lambda ps: torch.optim.AdamW(ps, lr=lr, weight_decay=0.0),
           "sgd": lambda ps: torch.optim.SGD(ps, lr=lr)}[opt_name](list(model.parameters()))
    factor, dsteps = decay
    for i in range(steps):
        grads = []
        for r in (1, 2):
            j = 2 * i + (r - 1)
            model.zero_grad()
            OF.cross_entropy(model(x[j * 32:(j + 1) * 32]), y[j * 32:(j + 1) * 32]).backward()
            grads.append([p.grad.clone() for p in model.parameters()])
        for p, g1, g2 in zip(model.parameters(), *grads):
            p.grad = (g1 + g2) * 0.5
        for g in opt.param_groups:
            g["lr"] = lr * factor ** (i // dsteps) if dsteps else lr
        opt.step()
    return torch.cat([p.detach().flatten() for p in model.parameters()])


@pytest.mark.parametrize("opt_name", ["adam", "adamw"])
def test_ps_master_adam_equals_single_process(opt_name):
    """PS mode applies the configured optimizer (TF SyncReplicas wraps Adam,
    distributed_train.py:160-173); 3 steps of 2-worker full sync == single-process torch Adam on the mean
    gradient."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_opt_job, 3, ({"optimizer": opt_name, "lr": 1e-3}, out, 3))
    ref = _reference_run(opt_name, 3, 1e-3)
    for r in res:
        # a handful of near-zero-gradient elements differ by < 3% of one lr step (Adam's m / (sqrt(v) + eps)
        # amplifies last-bit differences of the summation order there); everything else matches to 1e-6
        torch.testing.assert_close(r[1], ref, rtol=1e-5, atol=3e-5)
        assert (r[1] - ref).abs().gt(1e-6).sum() < 20


def test_ps_master_staircase_lr():
    """TF exponential_decay(staircase=True): lr * factor ** (step // decay_steps), applied by the master."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_opt_job, 3, ({"optimizer": "sgd", "lr": 0.1, "lr_decay_factor": 0.5, "decay_steps": 2},
                                     out, 5))
    assert [round(r["lr"], 6) for r in res[0][0]] == [0.1, 0.1, 0.05, 0.05, 0.025]
    ref = _reference_run("sgd", 5, 0.1, decay=(0.5, 2))
    torch.testing.assert_close(res[0][1], ref, rtol=1e-5, atol=1e-6)


def _ps_pipe_job(rank, world, cfg_kw, out_dir, steps):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ps import PSConfig, PSMaster, PSWorker
    torch.manual_seed(0)
    model = build_model("mlp_cpp", 10)
    x, y = _data()
    cfg = PSConfig(lr=0.05, max_steps=steps, out_dir=out_dir, bucket_cap_mb=0.5, first_bucket_mb=0.05, **cfg_kw)

    def batches():
        i = 0
        while True:
            j = 2 * i + (rank - 1)
            yield x[(j * 32) % 512:(j * 32) % 512 + 32], y[(j * 32) % 512:(j * 32) % 512 + 32]
            i += 1

    if rank == 0:
        role = PSMaster(model, cfg, torch.device("cpu"))
        role.train()
        info = {"nb": role.nb}
    else:
        role = PSWorker(model, cfg, torch.device("cpu"), OF.cross_entropy)
        role.train(batches())
        info = {"fwd": role.fwd_start, "land": role.landed}
    role.close()
    return info, torch.cat([p.detach().flatten() for p in model.parameters()])


def test_ps_layer_pipelined_weight_push():
    """the master pushes weights bucket by bucket in forward order and each worker module
    waits only for its own bucket (MPI_code worker_nn.h:66-70): with a slow link (40 ms between buckets) the
    first layer's forward starts before the last weight bucket lands; numerics equal the one-transfer push."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_pipe_job, 3, ({"comm_type": "Bcast", "push_delay_ms": 40.0}, out, 3))
    assert res[0][0]["nb"] >= 3
    for info, _ in res[1:]:
        for step, t_fwd in info["fwd"].items():
            land = info["land"][step]
            assert len(land) == res[0][0]["nb"]
            assert t_fwd < max(land.values()) - 0.02, (step, t_fwd, land)
    mono = run_world(_ps_pipe_job, 3, ({"comm_type": "Bcast", "pipelined_push": False}, out, 3))
    for a, b in zip(res, mono):
        assert torch.equal(a[1], b[1])
    asyn = run_world(_ps_pipe_job, 3, ({"comm_type": "Async", "push_delay_ms": 5.0}, out, 3))
    for a, b in zip(res, asyn):
        assert torch.equal(a[1], b[1])


def test_ps_master_checkpoints_by_time_and_final():
    """TF Supervisor(save_model_secs) + the chief's final save (distributed_train.py:215-223,346-350)."""
    out = tempfile.mkdtemp()
    ck = os.path.join(out, "ck")
    res = run_world(_ps_opt_job, 3, ({"optimizer": "adam", "lr": 1e-3, "checkpoint_dir": ck,
                                      "save_model_secs": 1e-6}, out, 3))
    files = sorted(os.listdir(ck))
    assert "checkpoint_final.pt" in files and "checkpoint_step1.pt" in files, files
    final = torch.load(os.path.join(ck, "checkpoint_final.pt"), weights_only=True)
    assert final["step"] == 3 and "optimizer" in final
    w = torch.cat([v.flatten() for k, v in final["state_dict"].items()])
    torch.testing.assert_close(w, res[0][1])


def test_ps_live_compute_times_in_master_log():
    """TF-04 live side channel: every worker's compute time reaches the master with its end-of-step marker."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_opt_job, 3, ({"log_compute_times": True}, out, 3))
    for r in res[0][0]:
        assert len(r["compute_ms"]) == 2 and all(v > 0 for v in r["compute_ms"])
        assert r["compute_ms"] == sorted(r["compute_ms"])


def _ps_fwd_kill_job(rank, world, out_dir, steps):
    import time
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ps import PSConfig, PSMaster, PSWorker
    torch.manual_seed(0)
    # layers called as modules, so forward pre-hooks can record which layers a step entered
    model = torch.nn.Sequential(torch.nn.Linear(784, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                                torch.nn.Linear(256, 256), torch.nn.ReLU(), torch.nn.Linear(256, 10))
    x, y = _data()
    cfg = PSConfig(num_aggregate=1, lr=0.05, max_steps=steps, out_dir=out_dir)
    entered = []                               # (step, layer) of every forward layer the worker started
    linears = [m for m in model.modules() if isinstance(m, torch.nn.Linear)]
    if rank == 0:
        role = PSMaster(model, cfg, torch.device("cpu"))
        out = role.train()
    else:
        role = PSWorker(model, cfg, torch.device("cpu"), OF.cross_entropy)
        if rank == 2:                          # the forward straggler: 0.3 s before each layer
            for i, m in enumerate(linears):
                m.register_forward_pre_hook(lambda mod, inp, i=i: (entered.append((role.cur, i)), time.sleep(0.3)) and None)

        def batches():
            i = 0
            while True:
                sl = slice((i * 32) % 512, (i * 32) % 512 + 32)
                yield x[sl], y[sl]
                i += 1
        role.train(batches())
        out = (role.compute_records, entered, len(linears))
    role.close()
    return out


def test_ps_worker_killed_mid_forward_stops_before_next_layer():
    """the C++ worker abandons the step before every FORWARD layer too (worker_nn.h:56-64).
    k = 1 of 2: rank 2 spends 0.3 s before each layer, rank 1 finishes the whole step first, the master kills
    rank 2, and rank 2 must stop before its next layer instead of finishing the forward."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_fwd_kill_job, 3, (out, 3), timeout=240)
    recs, entered, n_layers = res[2]
    killed = [r for r in recs if r["aborted"]]
    assert killed and all(r["abort_phase"] == "forward" for r in killed), recs
    for r in killed:
        layers = [i for s, i in entered if s == r["step"]]
        assert len(layers) <= 2 < n_layers, (r["step"], layers, n_layers)
    assert all(r["count"] == 1 and r["arrived"] == [1] for r in res[0])


def _ps_gather_job(rank, world, out_dir, steps):
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ps import PSConfig, run_ps
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(784, 1024), torch.nn.ReLU(), torch.nn.Linear(1024, 1024),
                                torch.nn.ReLU(), torch.nn.Linear(1024, 10))
    x, y = _data()
    cfg = PSConfig(lr=0.01, max_steps=steps, out_dir=out_dir, bucket_cap_mb=1.0, first_bucket_mb=0.25)

    def batches():
        while True:
            yield x[:32], y[:32]
    return run_ps(model, cfg, torch.device("cpu"), loss_fn=OF.cross_entropy, batches=batches())


def test_ps_master_receives_workers_concurrently():
    """the master posts each gradient receive the moment its arrival is announced (one
    staging slot per (worker, bucket)) instead of one blocking receive at a time into one buffer: with 8
    workers streaming ~7 MB each, the receives overlap -- the step's gather time is below the sum of the
    individual transfer times."""
    out = tempfile.mkdtemp()
    res = run_world(_ps_gather_job, 9, (out, 4), timeout=300)
    log = res[0]
    assert all(r["count"] == 8 for r in log)
    assert all(r["receives"] == 8 * len(r["bucket_counts"]) for r in log)
    overlapped = [r["xfer_ms_sum"] / r["gather_ms"] for r in log[1:]]
    assert max(overlapped) > 1.5, [(r["gather_ms"], r["xfer_ms_sum"]) for r in log]
