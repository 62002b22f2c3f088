"""Helpers to run a function in `world` CPU processes over gloo (the modern "mpirun -n N on one host",
SURVEY.md §4)."""
import faulthandler
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port():
    """A port that was free a moment ago (bind-and-close).  Only for launchers that must be given a port up
    front (torchrun's rendezvous endpoint); :func:`run_world` hosts its store itself instead."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def host_store():
    """The rendezvous TCPStore, hosted by the test process on a port the kernel assigns at bind time (nothing
    can already hold it), the way torchrun's agent hosts it for its workers
    (``TORCHELASTIC_USE_AGENT_STORE=True``: every rank, rank 0 included, connects as a client)."""
    import datetime
    import torch.distributed as dist
    return dist.TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False,
                         timeout=datetime.timedelta(seconds=300))


def _to_np(obj):
    import torch
    if isinstance(obj, torch.Tensor):
        return ("__tensor__", obj.detach().cpu().numpy().copy())
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_np(o) for o in obj)
    if isinstance(obj, dict):
        return {k: _to_np(v) for k, v in obj.items()}
    return obj


def _from_np(obj):
    import torch
    if isinstance(obj, tuple) and len(obj) == 2 and obj[0] == "__tensor__":
        return torch.from_numpy(obj[1])
    if isinstance(obj, (list, tuple)):
        return type(obj)(_from_np(o) for o in obj)
    if isinstance(obj, dict):
        return {k: _from_np(v) for k, v in obj.items()}
    return obj


def _entry(rank, world, port, fn, args, q, device="cpu", backend="gloo", env=None, timeout=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TORCHELASTIC_USE_AGENT_STORE="True", **(env or {}))
    if timeout:
        # a rank stuck past the parent's deadline prints every thread's Python stack to stderr and exits
        faulthandler.dump_traceback_later(max(5.0, timeout - 10.0), exit=True)
    try:
        import torch
        torch.set_num_threads(1)
        from pytorch_distributed_nn_amd.parallel import runtime
        runtime.init_process_group(backend=backend, device=device)
        res = fn(rank, world, *args)
        q.put((rank, "ok", _to_np(res)))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        try:
            from pytorch_distributed_nn_amd.parallel import runtime
            runtime.destroy()
        except Exception:
            pass


def run_world(fn, world=2, args=(), timeout=180, device="cpu", backend="gloo", env=None):
    """device="cpu": CPU tensors over gloo; device=None: every rank uses the (single) GPU, still over gloo
    (RCCL needs one GPU per rank; gloo moves GPU tensors through the host).  backend="nccl" with world=1
    and env={"PDNN_FORCE_PG": "1", ...} runs the RCCL path on a one-GPU box."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = host_store()          # kept alive (and its port held) until every rank has finished
    port = store.port
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q, device, backend, env, timeout))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{res}")
            out[rank] = _from_np(res)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        del store
    return [out[r] for r in range(world)]


def kofn_step(ddp, loss_fn):
    """One k-of-n DDP step: forward + loss (``loss_fn()``) and ``ddp.backward``.  True when this rank was cut
    short -- in its backward, or already in its forward (DDP.forward raises StepAborted after taking part in the
    step's collectives)."""
    from pytorch_distributed_nn_amd.parallel.ddp import StepAborted
    try:
        loss = loss_fn()
    except StepAborted:
        return True
    return ddp.backward(loss)
