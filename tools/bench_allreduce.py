"""Collective bandwidth sweep ("a bus-bandwidth sweep on 2/4/8 GPUs"; the reference
has no equivalent — its only comm test is the tagged p2p send of pytorch_code/comm_test.py:1-40).

One process per GPU, launched like bench.py::

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py
    python tools/bench_allreduce.py --world 2 --cpu          # gloo rehearsal on the CPU (spawns ranks itself)

For each message size it times ``iters`` back-to-back collectives (after ``warmup``) and reports, nccl-tests
style, ``algbw = bytes / t`` and ``busbw = algbw * factor`` with factor 2(n-1)/n for all_reduce and (n-1)/n
for reduce_scatter / all_gather (broadcast: 1).  busbw is the number to compare against the per-GPU xGMI
budget (7 links x ~153 GB/s per direction on MI355X): a ring all-reduce is bound by one link per hop, so
busbw far below ~7x153 GB/s at large sizes means RCCL is not spreading channels over all links.

The DDP bucket size (``bench.py --bucket-mb``, ``DistributedDataParallel(bucket_cap_mb=...)``) should sit
where this curve has flattened: below it a bucket pays latency, above it overlap with backward gets coarser.
Rank 0 prints one JSON line per (op, dtype, size).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FACTORS = {
    "all_reduce": lambda n: 2.0 * (n - 1) / n,
    "reduce_scatter": lambda n: (n - 1) / n,
    "all_gather": lambda n: (n - 1) / n,
    "broadcast": lambda n: 1.0,
}


def _sizes(lo: int, hi: int):
    s = lo
    while s <= hi:
        yield s
        s *= 4


def _one(op: str, nbytes: int, dtype, dev, world: int, iters: int, warmup: int, sync, reduce_op="avg"):
    n = max(world, nbytes // torch.tensor([], dtype=dtype).element_size())
    n -= n % world
    x = torch.ones(n, dtype=dtype, device=dev)
    out = torch.empty(n // world, dtype=dtype, device=dev)
    full = torch.empty(n, dtype=dtype, device=dev)
    # the DDP wrapper's op: AVG on RCCL (PreMulSum of 1/world -- a real reduction kernel even at world 1, where a
    # SUM is a no-op RCCL skips: the r3 sweep timed exactly that no-op), SUM on gloo
    rop = dist.ReduceOp.AVG if (reduce_op == "avg" and dev.type == "cuda") else dist.ReduceOp.SUM

    def run():
        if op == "all_reduce":
            dist.all_reduce(x, op=rop)
        elif op == "reduce_scatter":
            dist.reduce_scatter_tensor(out, x, op=rop)
        elif op == "all_gather":
            dist.all_gather_into_tensor(full, out)
        else:
            dist.broadcast(x, 0)

    for _ in range(warmup):
        run()
    sync()
    dist.barrier()
    if dev.type == "cuda":
        # device time of the collectives themselves: events on the current stream, which every RCCL launch joins
        # and waits on (the host's launch latency does not enter)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            run()
        e1.record()
        e1.synchronize()
        dt = e0.elapsed_time(e1) / 1e3 / iters
    else:
        t0 = time.perf_counter()
        for _ in range(iters):
            run()
        sync()
        dt = (time.perf_counter() - t0) / iters
    t = torch.tensor([dt], dtype=torch.float64)
    if dev.type == "cuda":
        t = t.to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    size = n * x.element_size()
    algbw = size / dt / 1e9
    return {"op": op, "reduce_op": reduce_op if op in ("all_reduce", "reduce_scatter") else None,
            "dtype": str(dtype).replace("torch.", ""), "bytes": size, "us": round(dt * 1e6, 2),
            "algbw_GBps": round(algbw, 2), "busbw_GBps": round(algbw * FACTORS[op](world), 2), "world": world}


def run(args):
    from pytorch_distributed_nn_amd.parallel import runtime
    env = runtime.init_process_group(device="cpu" if args.cpu else None)
    world = runtime.world_size()
    dev = torch.device("cpu") if args.cpu else runtime.device()
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    dtypes = [getattr(torch, d) for d in args.dtypes.split(",")]
    rows = []
    for op in args.ops.split(","):
        for dt in dtypes:
            for nb in _sizes(args.min_bytes, args.max_bytes):
                r = _one(op, nb, dt, dev, world, args.iters, args.warmup, sync, args.reduce_op)
                rows.append(r)
                if env.rank == 0:
                    print(json.dumps(r), flush=True)
    runtime.destroy()
    return rows


def _spawn_entry(rank, world, port, argv):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    run(argv)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather")
    ap.add_argument("--dtypes", default="float32,bfloat16")
    ap.add_argument("--min-bytes", type=int, default=64 * 1024)
    ap.add_argument("--max-bytes", type=int, default=256 * 2 ** 20)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reduce-op", default="avg", choices=["avg", "sum"],
                    help="reduction of all_reduce / reduce_scatter (avg = what DistributedDataParallel issues)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu", action="store_true", help="gloo on the CPU")
    ap.add_argument("--world", type=int, default=0, help="spawn this many local ranks (CPU rehearsal)")
    args = ap.parse_args(argv)
    if args.world > 1 and "RANK" not in os.environ:
        import socket
        import torch.multiprocessing as mp
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        mp.start_processes(_spawn_entry, args=(args.world, port, args), nprocs=args.world, start_method="spawn")
        return
    run(args)


if __name__ == "__main__":
    main()
