"""Trainer resume semantics (epoch-end checkpoints must resume at the NEXT epoch, mid-epoch
checkpoints after the steps already run) on CPU."""
import torch

from pytorch_distributed_nn_amd.trainer import Trainer


class _Loader:
    def __init__(self, n=3, bs=4):
        self.n, self.bs = n, bs

    def __len__(self):
        return self.n

    def __iter__(self):
        g = torch.Generator().manual_seed(0)
        while True:
            yield torch.randn(self.bs, 8, generator=g), torch.randint(0, 4, (self.bs,), generator=g)


def _trainer(ckdir, **kw):
    torch.manual_seed(0)
    m = torch.nn.Linear(8, 4)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    return Trainer(m, opt, loss_fn=torch.nn.functional.cross_entropy, checkpoint_dir=str(ckdir), log_interval=100,
                   printer=lambda *a: None, **kw)


def test_epoch_end_resume_runs_only_remaining_epochs(tmp_path):
    t = _trainer(tmp_path)
    t.train(_Loader(), epochs=2)
    assert t.step_no == 6
    t2 = _trainer(tmp_path)
    ck = t2.resume(str(tmp_path / "checkpoint_ep1.pt"))
    assert ck["epoch"] == 2 and t2.step_no == 6
    t2.train(_Loader(), epochs=3)
    assert t2.step_no == 9                      # exactly one more epoch, not a repeat of epoch 1
    assert [r["epoch"] for r in t2.history] == [2, 2, 2]


def test_mid_epoch_resume_continues_inside_the_epoch(tmp_path):
    t = _trainer(tmp_path, checkpoint_interval=2)
    t.train(_Loader(), epochs=5, max_steps=5)
    t2 = _trainer(tmp_path)
    ck = t2.resume("auto")
    assert ck["step"] == 4 and ck["epoch"] == 1   # newest: checkpoint_step4 (epoch 1 in progress)
    t2.train(_Loader(), epochs=2)
    assert t2.step_no == 6                       # steps 5 and 6 complete epoch 1
    assert [r["epoch"] for r in t2.history] == [1, 1]


def test_resume_restores_weights(tmp_path):
    t = _trainer(tmp_path)
    t.train(_Loader(), epochs=1)
    w = t.model.weight.detach().clone()
    t2 = _trainer(tmp_path)
    t2.resume("auto")
    assert torch.equal(t2.model.weight, w)


class _EpochLoader(_Loader):
    """Per-epoch reshuffled stream (like data.DataLoader): a fresh iterator restarts at epoch 0's order."""

    def __iter__(self):
        data = torch.randn(self.n * self.bs, 8, generator=torch.Generator().manual_seed(1))
        lab = torch.arange(self.n * self.bs) % 4
        g = torch.Generator().manual_seed(2)
        while True:
            perm = torch.randperm(self.n * self.bs, generator=g)
            for i in range(self.n):
                idx = perm[i * self.bs:(i + 1) * self.bs]
                yield data[idx], lab[idx]


def test_resume_in_later_epoch_sees_the_uninterrupted_batches(tmp_path):
    # a resume in epoch >= 1 must train on that epoch's order (not epoch 0's) and skip exactly the
    # batches already consumed; the resumed run then ends bit-identical to the uninterrupted one
    t = _trainer(tmp_path, checkpoint_interval=4)
    t.train(_EpochLoader(), epochs=3)
    ref = t.model.weight.detach().clone()
    t2 = _trainer(tmp_path)
    ck = t2.resume(str(tmp_path / "checkpoint_step4.pt"))
    assert ck["step"] == 4 and ck["epoch"] == 1
    t2.train(_EpochLoader(), epochs=3)
    assert t2.step_no == 9
    assert torch.equal(t2.model.weight, ref)


def test_resume_at_large_step_fast_forwards_without_building_batches(tmp_path):
    """resuming at step 20,000 must not decode / transform / copy 20,000 batches (the loader skips its
    sampler), and a short hang watchdog started before train() must not fire during the fast-forward."""
    import time

    import numpy as np

    from pytorch_distributed_nn_amd.data.datasets import DataLoader, DataSet
    from pytorch_distributed_nn_amd.parallel.watchdog import CommWatchdog
    built = []

    def slow_transform(x):          # ~2 ms per built batch: 20,000 of them would take 40 s
        built.append(1)
        time.sleep(0.002)
        return x

    rng = np.random.RandomState(0)
    ds = DataSet(rng.randn(64, 8).astype(np.float32), rng.randint(0, 4, 64))
    loader = DataLoader(ds, 4, transform=slow_transform)
    fired = []
    # 3 s: a cold first import inside train() can take over a second on a loaded host; building the 20,000
    # skipped batches would take ~40 s
    wd = CommWatchdog(timeout_s=3.0, rank=0, exit_on_hang=False, on_hang=fired.append, poll_s=0.05).start()
    t = _trainer(tmp_path, watchdog=wd)
    t.step_no = 20000
    t0 = time.perf_counter()
    t.train(loader, epochs=10 ** 6, steps_per_epoch=16, max_steps=20003)
    wd.stop()
    loader.close()
    assert t.step_no == 20003 and not fired
    assert time.perf_counter() - t0 < 5.0 and len(built) < 50
