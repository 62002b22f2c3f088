"""DDP on CPU/gloo at world_size 2 (BASELINE.json config 1; SURVEY.md §7.4 tests/cpu_gloo)."""
import torch

from dist_utils import kofn_step, run_world


def _ddp_vs_single(rank, world, model_name, shape, comm_dtype):
    import torch.distributed as dist
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(100 + rank)                     # different init per rank: broadcast must fix it
    m = build_model(model_name, 10)
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.5, first_bucket_cap_mb=0.05,
                                  comm_dtype=comm_dtype)
    # every rank holds rank 0's weights after the init broadcast
    ref_state = {k: v.clone() for k, v in m.state_dict().items()}
    gathered = [torch.zeros_like(m.fc1.weight if hasattr(m, "fc1") else m.fc0.weight) for _ in range(world)]
    dist.all_gather(gathered, (m.fc1.weight if hasattr(m, "fc1") else m.fc0.weight).detach().contiguous())
    assert torch.equal(gathered[0], gathered[1])
    g = torch.Generator().manual_seed(7)
    x = torch.randn(world * 4, *shape, generator=g)
    y = torch.randint(0, 10, (world * 4,), generator=g)
    ddp.zero_grad()
    loss = OF.cross_entropy(ddp(x[rank * 4:(rank + 1) * 4]), y[rank * 4:(rank + 1) * 4])
    loss.backward()
    grads = {n: p.grad.clone() for n, p in m.named_parameters()}
    # single-process reference on the concatenated global batch
    single = build_model(model_name, 10)
    single.load_state_dict(ref_state)
    lg = OF.cross_entropy(single(x), y)
    lg.backward()
    tol = 2e-2 if comm_dtype is not None else 1e-5
    for n, p in single.named_parameters():
        err = (grads[n] - p.grad).abs().max().item() / max(p.grad.abs().max().item(), 1e-8)
        assert err < tol, (n, err)
    return ddp.bucket_sizes_mb()


def test_ddp_matches_single_process_mlp():
    sizes = run_world(_ddp_vs_single, 2, ("mlp2", (784,), None))
    assert sizes[0] == sizes[1]
    assert len(sizes[0]) >= 2
    assert sizes[0][0] <= 0.6          # small first bucket so comm starts early


def test_ddp_matches_single_process_lenet():
    run_world(_ddp_vs_single, 2, ("LeNet", (1, 28, 28), None))


def test_ddp_bf16_wire_compression():
    run_world(_ddp_vs_single, 2, ("mlp2", (784,), torch.bfloat16))


def _bucket_order(rank, world):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    m = build_model("mlp_cpp", 10)
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.5, first_bucket_cap_mb=0.01)
    params = ddp.flat.params
    # bucket 0 holds the LAST parameters (gradients arrive in reverse order)
    first = [i for i, p in enumerate(params) if ddp._pbucket[id(p)] == 0]
    assert max(first) == len(params) - 1
    last = [i for i, p in enumerate(params) if ddp._pbucket[id(p)] == len(ddp.buckets) - 1]
    assert min(last) == 0
    return len(ddp.buckets)


def test_bucket_reverse_order():
    n = run_world(_bucket_order, 2)
    assert n[0] > 2


def _no_sync(rank, world):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(0)
    m = build_model("mlp2", 10)
    ddp = DistributedDataParallel(m)
    x = torch.randn(8, 784) + rank
    y = torch.randint(0, 10, (8,))
    ddp.zero_grad()
    with ddp.no_sync():
        OF.cross_entropy(ddp(x), y).backward()
    local = m.fc0.weight.grad.clone()
    OF.cross_entropy(ddp(x), y).backward()      # synced step: average of (2*local) over ranks
    return local, m.fc0.weight.grad.clone()


def test_no_sync_accumulates_locally():
    (l0, s0), (l1, s1) = run_world(_no_sync, 2)
    assert not torch.allclose(l0, l1)
    assert torch.allclose(s0, s1, atol=1e-6)
    assert torch.allclose(s0, (2 * l0 + 2 * l1) / 2, atol=1e-5)


def _straggler(rank, world):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(0)
    m = build_model("mlp2", 10)
    ddp = DistributedDataParallel(m, straggler_mode=True)
    ddp.attach_optimizer(SGD(m.parameters(), lr=1.0))
    x = torch.randn(8, 784) * (rank + 1)
    y = torch.randint(0, 10, (8,))
    ddp.set_alive(rank == 0)                   # rank 1 is "killed" this step
    ddp.zero_grad()
    OF.cross_entropy(ddp(x), y).backward()
    return m.fc0.weight.grad.clone(), ddp.last_counts.clone(), x, y


def test_straggler_count_correct_average():
    """Manual drop (set_alive): sum of alive grads / per-bucket alive count (fixes reference defect D3)."""
    (g0, c0, x0, y0), (g1, c1, _, _) = run_world(_straggler, 2)
    assert torch.equal(c0, c1) and torch.all(c0 == 1)
    assert torch.allclose(g0, g1)
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    torch.manual_seed(0)
    m = build_model("mlp2", 10)
    OF.cross_entropy(m(x0), y0).backward()
    assert torch.allclose(g0, m.fc0.weight.grad, atol=1e-6)


def _kofn(rank, world, k, sleep_ms, steps):
    """k-of-n in collective form: the slowest rank (world-1) sleeps per parameter in its backward."""
    import time
    import torch.distributed as dist
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(0)
    m = build_model("mlp_cpp", 10)
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.5, first_bucket_cap_mb=0.05, num_aggregate=k)
    ref = build_model("mlp_cpp", 10)
    if rank == world - 1 and sleep_ms:
        for p in m.parameters():
            p.register_post_accumulate_grad_hook(lambda _p: time.sleep(sleep_ms / 1e3))
    res = []
    for step in range(steps):
        g = torch.Generator().manual_seed(10 * step + rank)
        x, y = torch.randn(16, 784, generator=g), torch.randint(0, 10, (16,), generator=g)
        # this rank's own full gradient (reference for the count-correct average)
        ref.load_state_dict(m.state_dict())
        ref.zero_grad()
        OF.cross_entropy(ref(x), y).backward()
        local = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
        ddp.zero_grad()
        t0 = time.perf_counter()
        aborted = kofn_step(ddp, lambda: OF.cross_entropy(ddp(x), y))
        dt = time.perf_counter() - t0
        contrib = torch.tensor(ddp.last_contrib)
        # expected: per bucket, the mean over the ranks that contributed real gradients
        locs = [torch.zeros_like(local) for _ in range(world)]
        cons = [torch.zeros_like(contrib) for _ in range(world)]
        dist.all_gather(locs, local)
        dist.all_gather(cons, contrib)
        got = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
        exp = torch.zeros_like(local)
        flat_order = ddp.flat.params
        offs = {}
        o = 0
        for p in m.parameters():
            offs[id(p)] = (o, o + p.numel())
            o += p.numel()
        for bi, (s, e, _) in enumerate(ddp.buckets):
            cnt = sum(float(c[bi]) for c in cons)
            for p in flat_order:
                if ddp._pbucket[id(p)] != bi:
                    continue
                a, b = offs[id(p)]
                tot = sum(locs[r][a:b] * float(cons[r][bi]) for r in range(world))
                exp[a:b] = tot / max(cnt, 1.0)
        err = float((got - exp).abs().max() / exp.abs().max().clamp_min(1e-12))
        res.append((aborted, dt, err, [float(v) for v in ddp.last_counts]))
    ddp.close()
    return res


def test_kofn_kill_straggler_short_circuits_and_averages_by_count():
    """World 4, k = 3: rank 3 sleeps 40 ms per parameter (16 parameters: a 640 ms backward).  Once three
    ranks finished, rank 3 abandons its backward; every bucket is averaged over the ranks that sent real
    gradients for it."""
    out = run_world(_kofn, 4, (3, 40.0, 3), timeout=240)
    slow = out[3]
    assert all(a for a, _, _, _ in slow), slow                   # short-circuited every step
    # far below the 0.64 s full backward (step 0 pays gloo's lazy connection setup on the fast ranks; the
    # margin leaves room for a loaded CI host, where 0.2 s against a 0.32 s backward flaked)
    assert max(dt for _, dt, _, _ in slow[1:]) < 0.45, slow
    for r in range(4):
        for aborted, dt, err, counts in out[r]:
            assert err < 1e-5, (r, err)
            assert min(counts) >= 3 and max(counts) <= 4
    assert all(not a for a, _, _, _ in out[0])


def test_kofn_full_participation_matches_plain_average():
    """k = n: nobody is killed; the result equals the plain average."""
    out = run_world(_kofn, 2, (2, 0.0, 2))
    for r in range(2):
        for aborted, dt, err, counts in out[r]:
            assert not aborted and err < 1e-5 and counts == [2.0] * len(counts)


def _deadline(rank, world):
    import time
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(0)
    m = build_model("mlp_cpp", 10)
    # k = n (wait for everyone) but a 60 ms step deadline: the backup-worker / interval form
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.5, first_bucket_cap_mb=0.05, deadline_ms=60.0)
    if rank == 1:
        for p in m.parameters():
            p.register_post_accumulate_grad_hook(lambda _p: time.sleep(0.02))
    res = []
    for step in range(3):
        x, y = torch.randn(16, 784), torch.randint(0, 10, (16,))
        ddp.zero_grad()
        t0 = time.perf_counter()
        aborted = kofn_step(ddp, lambda: OF.cross_entropy(ddp(x), y))
        res.append((aborted, time.perf_counter() - t0, [float(v) for v in ddp.last_counts]))
    ddp.close()
    return res


def test_ddp_step_deadline_drops_late_rank():
    out = run_world(_deadline, 2)
    for aborted, dt, counts in out[1][1:]:
        assert aborted and dt < 0.25, out[1]            # 16 x 20 ms = 0.32 s without the deadline
        assert min(counts) >= 1 and max(counts) <= 2
    assert not any(a for a, _, _ in out[0])


def _deadline_after_fast_steps(rank, world):
    import time
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(0)
    m = build_model("mlp2", 10)
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.5, first_bucket_cap_mb=0.05, deadline_ms=120.0)
    slow = {"on": False}
    if rank == 1:
        for p in m.parameters():
            p.register_post_accumulate_grad_hook(lambda _p: time.sleep(0.4) if slow["on"] else None)
    res = []
    for step in range(26):
        slow["on"] = step == 25
        x, y = torch.randn(8, 784), torch.randint(0, 10, (8,))
        ddp.zero_grad()
        t0 = time.perf_counter()
        aborted = kofn_step(ddp, lambda: OF.cross_entropy(ddp(x), y))
        res.append((aborted, time.perf_counter() - t0))
    ddp.close()
    return res


def test_ddp_deadline_fires_on_time_after_many_fast_steps():
    """25 steps that finish well inside the 120 ms deadline, then one slow step on rank 1.  The
    deadline thread must close the slow step ~120 ms after it began (it used to walk the backlog of fast
    steps one deadline each and fire seconds late)."""
    out = run_world(_deadline_after_fast_steps, 2)
    aborted, dt = out[1][-1]
    assert aborted and dt < 0.5, out[1][-3:]          # 4 params x 0.4 s = 1.6 s without the deadline
    assert not any(a for a, _ in out[1][:-1])


def _world4_consistency(rank, world):
    """Fused-backward DDP at world 4: after the all-reduce every rank holds BIT-identical gradients,
    buckets launch in the same order everywhere, and BN running statistics stay identical (buffers are
    broadcast from rank 0 every forward, data_parallel_dist.py:133-138)."""
    import torch.distributed as dist
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(rank)
    m = build_model("resnet18", 10)
    ddp = DistributedDataParallel(m, bucket_cap_mb=4.0, first_bucket_cap_mb=0.25)
    opt = SGD(m.parameters(), lr=0.05, momentum=0.9)
    orders = []
    for step in range(2):
        g = torch.Generator().manual_seed(100 * step + rank)       # different data per rank
        x, y = torch.randn(4, 3, 32, 32, generator=g), torch.randint(0, 10, (4,), generator=g)
        opt.zero_grad()
        OF.cross_entropy(ddp(x), y).backward()
        grads = ddp.flat.grad.clone()
        allg = [torch.empty_like(grads) for _ in range(world)]
        dist.all_gather(allg, grads)
        for r in range(world):
            assert torch.equal(allg[r], allg[0]), (step, r)
        orders.append(ddp.last_launch_order)
        opt.step()
    ddp.sync_buffers()
    bufs = torch.cat([b.float().reshape(-1) for b in m.buffers()])
    allb = [torch.empty_like(bufs) for _ in range(world)]
    dist.all_gather(allb, bufs)
    return orders, all(torch.equal(b, allb[0]) for b in allb), len(ddp.buckets)


def test_world4_bit_identical_grads_and_launch_order():
    out = run_world(_world4_consistency, 4, timeout=300)
    orders0, same_bufs, nb = out[0]
    assert nb >= 3 and same_bufs
    for orders, _, _ in out:
        assert orders == orders0
        assert all(o == list(range(nb)) for o in orders)           # strictly in bucket order


def _kofn_fwd(rank, world):
    import time
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel, StepAborted
    def net():
        torch.manual_seed(0)     # layers called as modules: forward pre-hooks record the layers a step entered
        return torch.nn.Sequential(torch.nn.Linear(784, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256),
                                   torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                                   torch.nn.Linear(256, 10))
    m, ref = net(), net()
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.5, first_bucket_cap_mb=0.05, num_aggregate=1)
    linears = [mod for mod in m.modules() if isinstance(mod, torch.nn.Linear)]
    entered = []
    if rank == 1:                          # a slow FORWARD: 0.3 s before each layer
        for i, mod in enumerate(linears):
            mod.register_forward_pre_hook(lambda _m, _i, i=i: (entered.append((ddp.step + 1, i)), time.sleep(0.3)) and None)
    res = []
    for step in range(2):
        g = torch.Generator().manual_seed(100 + step)
        x, y = torch.randn(16, 784, generator=g), torch.randint(0, 10, (16,), generator=g)
        ref.load_state_dict({k.replace("module.", ""): v for k, v in m.state_dict().items()})
        ref.zero_grad()
        OF.cross_entropy(ref(x), y).backward()
        local0 = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])   # rank 0's gradient (same batch)
        ddp.zero_grad()
        try:
            aborted = ddp.backward(OF.cross_entropy(ddp(x), y))
        except StepAborted:
            aborted = "forward"
        got = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
        err = float((got - local0).abs().max() / local0.abs().max())
        layers = [i for s, i in entered if s == ddp.step]
        res.append((aborted, ddp.abort_phase, [float(v) for v in ddp.last_counts], err, len(layers), len(linears)))
    ddp.close()
    return res


def test_kofn_rank_killed_in_forward_stops_before_next_layer():
    """k = 1 of 2, rank 1's forward is slow (0.3 s per layer).  Rank 0 finishes and closes the
    step; rank 1 abandons its FORWARD before the next layer (not only its backward), takes part in the step's
    collectives with zero buckets, and both ranks end with rank 0's gradient (every bucket count 1)."""
    out = run_world(_kofn_fwd, 2, (), timeout=240)
    for r in range(2):
        for aborted, phase, counts, err, n_entered, n_layers in out[r]:
            assert counts == [1.0] * len(counts) and err < 1e-5, out[r]
    for aborted, phase, counts, err, n_entered, n_layers in out[1]:
        assert aborted == "forward" and phase == "forward" and n_entered <= 2 < n_layers, out[1]
    assert all(a is False for a, *_ in out[0])


def _bn_buffers_at_forward(rank, world):
    """Buffers seen by every training forward, recorded by a pre-hook on the wrapped module (after DDP.forward has
    made them rank 0's): identical on all ranks at every step, although each rank's own forward moves them with its
    own batch.  From the second forward on they come from the broadcast issued at the end of the previous backward."""
    import torch.distributed as dist
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(rank)
    m = build_model("resnet18", 10)
    ddp = DistributedDataParallel(m, bucket_cap_mb=4.0, first_bucket_cap_mb=0.25)
    opt = SGD(m.parameters(), lr=0.05, momentum=0.9)
    seen, pre_issued = [], []
    m.register_forward_pre_hook(lambda mod, inp: seen.append(torch.cat([b.float().reshape(-1) for b in mod.buffers()])))
    for step in range(4):
        g = torch.Generator().manual_seed(100 * step + rank)
        x, y = torch.randn(4, 3, 32, 32, generator=g), torch.randint(0, 10, (4,), generator=g)
        pre_issued.append(ddp._bn_work is not None)
        opt.zero_grad()
        OF.cross_entropy(ddp(x), y).backward()
        opt.step()
    same = []
    for v in seen:
        allv = [torch.empty_like(v) for _ in range(world)]
        dist.all_gather(allv, v)
        same.append(all(torch.equal(a, allv[0]) for a in allv))
    moved = not torch.equal(seen[0], seen[-1])
    return same, pre_issued, moved


def test_bn_buffer_broadcast_issued_after_backward_keeps_every_forward_semantics():
    """the BN-buffer broadcast leaves the start of the step (issued behind the last bucket of
    the previous backward) but every training forward still starts from rank 0's buffers
    (data_parallel_dist.py:133-138)."""
    out = run_world(_bn_buffers_at_forward, 2)
    for same, pre, moved in out:
        assert all(same) and moved
        assert pre == [False, True, True, True]


def _ovl_predicate(rank, world):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    m = build_model("mlp2", 10)
    avg = DistributedDataParallel(m, bucket_cap_mb=0.5)
    # gloo reduces with SUM and divides by the world size only after every wait: a bucket is not final when its
    # collective completes, so per-bucket optimizer updates (overlap_optimizer) must stay off
    assert not avg.nccl and avg.world == 2
    assert not avg._ovl_reduced_is_final()
    m2 = build_model("mlp2", 10)
    summed = DistributedDataParallel(m2, bucket_cap_mb=0.5, average=False)
    assert summed._ovl_reduced_is_final()
    return True


def test_overlap_optimizer_never_consumes_unaveraged_gloo_buckets():
    assert all(run_world(_ovl_predicate, 2))
