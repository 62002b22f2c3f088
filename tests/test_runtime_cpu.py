"""C++ host runtime (csrc/runtime/) tests: control-plane store, PS coordinator semantics, IDX reader,
native MLP trainer and its master/evaluator/worker roles (the reference's MPI_code stack)."""
import multiprocessing as mp
import os
import threading
import time

import numpy as np
import pytest

from pytorch_distributed_nn_amd.utils import native as N


def test_store_basic_and_blocking_get():
    srv = N.StoreServer(0)
    try:
        a, b = N.Store("127.0.0.1", srv.port), N.Store("127.0.0.1", srv.port)
        a.set("k", b"hello")
        assert b.get("k") == b"hello"
        assert b.check("k") and not b.check("nope")
        assert a.add("cnt", 2) == 2 and b.add("cnt", 3) == 5
        with pytest.raises(N.StoreTimeout):
            b.get("later", timeout_ms=50)
        got = {}

        def waiter():
            got["v"] = b.get("later", timeout_ms=5000)
        t = threading.Thread(target=waiter)
        t.start()
        time.sleep(0.05)
        a.set("later", "x" * 1000)
        t.join(5)
        assert got["v"] == b"x" * 1000
        a.set_int("step", 42)
        assert b.get_int("step") == 42
        a.set("kill/3/1", b"1")
        a.set("kill/3/2", b"1")
        assert sorted(b.keys("kill/3/")) == ["kill/3/1", "kill/3/2"]
        a.delete("k")
        assert not b.check("k")
        # PUSH: queue append in one round trip, numbered like add("q_n") + set("q/<n>")
        assert a.push("q", "0,1,2") == 1 and b.push("q", b"3,4,5") == 2
        assert a.get("q/1") == b"0,1,2" and a.get("q/2") == b"3,4,5" and a.get_int("q_n") == 2
        big = np.random.rand(1 << 18).astype(np.float32)
        a.set("big", big)
        assert np.array_equal(np.frombuffer(b.get("big"), np.float32), big)
        a.close()
        b.close()
    finally:
        srv.stop()


def test_ps_full_sync_and_duplicates():
    ps = N.PSCoordinator(n_workers=3, n_layers=2)
    ps.begin_step(5)
    assert ps.offer(0, 0, 5) == ps.ACCEPTED
    assert ps.offer(0, 0, 5) == ps.DUPLICATE          # ANY_SOURCE slot race (D2) cannot double count
    assert ps.offer(1, 0, 4) == ps.STALE              # older step dropped (CPP-03 stale drop)
    assert ps.stale_dropped == 1
    for w in range(3):
        ps.offer(w, 1, 5)
    assert not ps.done()
    ps.offer(1, 0, 5)
    ps.offer(2, 0, 5)
    assert ps.done() and ps.count(0) == 3


def test_ps_k_of_n_kill():
    ps = N.PSCoordinator(n_workers=5, n_layers=4, kill_k=3)
    ps.begin_step(1)
    for w in (4, 0, 2):                                # arrival order of the sentinel layer 0
        for l in (3, 2, 1, 0):
            ps.offer(w, l, 1)
    ps.offer(1, 3, 1)                                  # worker 1 is half-way through its backward
    assert ps.done()
    assert ps.stragglers(0) == [1, 3]
    assert ps.count(0) == 3 and ps.count(3) == 4       # real per-layer counts for the average (fix D3)
    assert ps.offer(3, 0, 1) == ps.CLOSED
    tl = ps.timeline()
    assert len(tl) == 13 and tl[0][2] == 4


def test_ps_backup_workers():
    ps = N.PSCoordinator(n_workers=6, n_layers=3, n_to_collect=2)
    ps.begin_step(7)
    for l in range(3):
        ps.offer(l, l, 7)
    assert not ps.done()
    for l in range(3):
        ps.offer(5, l, 7)
    assert ps.done()


def test_idx_roundtrip(tmp_path):
    imgs = (np.random.rand(10, 28, 28) * 255).astype(np.uint8)
    labels = np.arange(10, dtype=np.uint8)
    N.idx_write(tmp_path / "img.idx", imgs)
    N.idx_write(tmp_path / "lab.idx", labels)
    assert np.array_equal(N.idx_read(tmp_path / "img.idx"), imgs)
    assert np.array_equal(N.idx_read(tmp_path / "lab.idx"), labels)
    # header is the big-endian magic of the MNIST files (mnist.h:36-86): 2051 for 3-D u8 images
    raw = open(tmp_path / "img.idx", "rb").read(4)
    assert int.from_bytes(raw, "big") == 2051
    idx = N.shuffle_indices(100, 66478)
    assert sorted(idx.tolist()) == list(range(100)) and idx.tolist() != list(range(100))


def _synthetic(n=2048, d=64, classes=10, seed=0):
    rng = np.random.default_rng(seed)
    centers = rng.normal(0, 1, (classes, d)).astype(np.float32)
    y = rng.integers(0, classes, n).astype(np.int32)
    x = centers[y] + 0.3 * rng.normal(0, 1, (n, d)).astype(np.float32)
    return x, y


def test_native_mlp_gradients_match_numpy():
    x, y = _synthetic(64, 16, 4)
    m = N.NativeMLP([16, 12, 4], batch=64, lr=0.5)
    W0, W1 = m.weights(0).copy(), m.weights(1).copy()
    m.forward_backward(x, y)
    # numpy reference of the bias-folded forward/backward
    z0 = np.concatenate([x, np.ones((64, 1), np.float32)], 1)
    h = 1 / (1 + np.exp(-(z0 @ W0)))
    z1 = np.concatenate([h, np.ones((64, 1), np.float32)], 1)
    s = z1 @ W1
    p = np.exp(s - s.max(1, keepdims=True))
    p /= p.sum(1, keepdims=True)
    d2 = (p - np.eye(4, dtype=np.float32)[y]) / 64
    g1 = z1.T @ d2
    d1 = (d2 @ W1[:-1].T) * h * (1 - h)
    g0 = z0.T @ d1
    assert np.allclose(m.grads(1), g1, atol=1e-5)
    assert np.allclose(m.grads(0), g0, atol=1e-5)


def test_native_mlp_single_machine_learns():
    x, y = _synthetic()
    m = N.NativeMLP([64, 32, 10], batch=128, lr=0.5)
    l0, e0 = m.evaluate(x, y)
    losses = m.train(x, y, 200)
    l1, e1 = m.evaluate(x, y)
    assert l1 < 0.5 * l0 and e1 < 0.2 and losses[-1] < losses[0]


def _role(role, port, rank, nprocs, ncollect, iters, out):
    x, y = _synthetic()
    rc = N.run_native_role(role, "127.0.0.1", port, rank, nprocs, ncollect, iters, x, y, [64, 32, 10], batch=64,
                           lr=0.5, shortcircuit=True, out_prefix=out)
    assert rc == 0, rc


def test_native_ps_backup_workers_with_evaluator(tmp_path):
    """master + evaluator + 4 workers, collect 2 per step (CPP-01: n_to_collect = n_procs - 2 - ...)."""
    srv = N.StoreServer(0)
    out = str(tmp_path) + "/"
    nprocs, ncollect, iters = 6, 2, 30
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_role, args=("master", srv.port, 0, nprocs, ncollect, iters, out))]
    ps.append(ctx.Process(target=_role, args=("evaluator", srv.port, 1, nprocs, ncollect, iters, out)))
    workers = [ctx.Process(target=_role, args=("worker", srv.port, r, nprocs, ncollect, iters, out))
               for r in range(2, nprocs)]
    try:
        for p in ps:
            p.start()
        # the evaluator scores the newest model it finds: start the workers only once it is connected (its
        # output file is open), or under load the whole run can finish first and leave it one row to write
        deadline = time.time() + 60
        while not any(f.startswith("time_loss_out_") for f in os.listdir(tmp_path)) and time.time() < deadline:
            time.sleep(0.05)
        for p in workers:
            p.start()
        ps += workers
        for p in ps:
            p.join(120)
            assert p.exitcode == 0
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()
        srv.stop()
    files = os.listdir(tmp_path)
    tl = [f for f in files if f.startswith("time_loss_out_SyncReplicasWithBackup2_4")]
    assert tl, files
    rows = [l.split() for l in open(tmp_path / tl[0]).read().strip().splitlines()]
    assert len(rows) >= 2
    first, last = float(rows[0][2]), float(rows[-1][2])
    assert last < first, (first, last)
    assert any(f.startswith("timeline_out_") for f in files)
