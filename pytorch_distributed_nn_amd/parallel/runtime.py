"""Process bootstrap: rank / world / local rank from torchrun *or* mpirun environments, device binding
and process-group init (torchrun-compatible env with an OMPI_COMM_WORLD_* fallback so
``mpirun -n N python ...`` launches — the reference's launch style, pytorch_code/README.md:8-11 —
still work).

One process per GPU.  On GPUs the backend is ``nccl`` (= RCCL on ROCm, over xGMI inside a node);
on CPU it is ``gloo`` (BASELINE.json config 1: CPU plumbing at world_size 2).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    master_addr: str = "127.0.0.1"
    master_port: int = 29500

    @property
    def is_master(self):
        return self.rank == 0


def _first(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            return v
    return default


def read_env() -> DistEnv:
    rank = int(_first("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "SLURM_PROCID", default=0))
    world = int(_first("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS", default=1))
    local = int(_first("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "SLURM_LOCALID", default=0))
    lws = int(_first("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", default=world))
    addr = _first("MASTER_ADDR", default="127.0.0.1")
    port = int(_first("MASTER_PORT", default=29500))
    return DistEnv(rank, world, local, lws, addr, port)


_ENV: DistEnv | None = None


def init_process_group(backend: str | None = None, device: str | None = None, timeout_s: float = 600.0) -> DistEnv:
    """Initialise torch.distributed from the environment (idempotent).  Returns the :class:`DistEnv`.

    ``backend=None`` picks nccl(RCCL) when a GPU is visible and ``device`` is not "cpu", else gloo.
    A single-process run (WORLD_SIZE unset or 1) skips process-group creation entirely."""
    global _ENV
    env = read_env()
    use_gpu = (device != "cpu") and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(env.local_rank % max(1, torch.cuda.device_count()))
    # PDNN_FORCE_PG=1: build the (RCCL) process group even for one rank, so a 1-GPU box can rehearse the
    # multi-GPU code path (DDP hooks + RCCL kernels on their stream) that the 8-GPU node runs
    force = os.environ.get("PDNN_FORCE_PG") == "1"
    if (env.world_size > 1 or force) and not dist.is_initialized():
        if env.world_size > 1:
            os.environ.setdefault("MASTER_ADDR", env.master_addr)
            os.environ.setdefault("MASTER_PORT", str(env.master_port))
        # dmabuf IPC is the only mode the box's driver supports (see task environment notes)
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        be = backend or ("nccl" if use_gpu else "gloo")
        kw = dict(backend=be, rank=env.rank, world_size=env.world_size,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        restart = os.environ.get("TORCHELASTIC_RESTART_COUNT")
        if env.world_size == 1 and "MASTER_PORT" not in os.environ:
            # a one-rank group (PDNN_FORCE_PG) needs no rendezvous: an in-process store, no port
            kw["store"] = dist.HashStore()
        elif restart not in (None, "", "0"):
            # a restarted worker group (parallel/watchdog.py) may share the launcher's store with the failed
            # attempt: namespace this attempt's keys so no rank reads a dead peer's address
            store, _, _ = next(dist.rendezvous("env://", env.rank, env.world_size,
                                               timeout=datetime.timedelta(seconds=timeout_s)))
            kw["store"] = dist.PrefixStore(f"pdnn_attempt{restart}", store)
        dist.init_process_group(**kw)
    _ENV = env
    return env


def get_env() -> DistEnv:
    return _ENV or read_env()


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def barrier():
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def destroy():
    if dist.is_initialized():
        dist.destroy_process_group()
