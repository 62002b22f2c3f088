"""Headline benchmark (BASELINE.json): samples/sec of ResNet-50 DDP training on 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--model resnet50|gpt2_small]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU (RCCL over xGMI for N > 1).  Model: ResNet-50, ImageNet layout (224x224x3 input,
1000 classes), random init; data: synthetic device-resident tensors of that shape.  Compute dtype bf16
(NHWC activations, fp32 accumulation, fp32 master weights / BN statistics / gradients), optimizer:
fused SGD with momentum 0.9 + weight decay, full step timed (forward, backward, bucketed all-reduce,
optimizer).  Per-GPU batch is fixed as N grows (weak scaling).  Rank 0 prints one JSON line with the
WHOLE-JOB samples/sec (max step time over ranks).  Every N runs the DDP code path: at N = 1 the wrapper's
bucket hooks all-reduce every bucket over a one-rank RCCL process group (BASELINE config 2, "DDP
world_size=1"), and the plain single-GPU step is measured in a second process and reported beside it
(``plain_step_1gpu``).

``--model gpt2_small`` benchmarks BASELINE.json config 4 instead: GPT-2 small (124M, T=1024, vocab
50304), per-GPU batch 8 sequences, fused AdamW, metric tokens/sec (whole node).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

STOCK_PYTORCH_1GPU = 6629.4   # profiles/stock_pytorch_resnet50.jsonl: torch autocast-bf16 channels_last, bs256


def native_loaded():
    """In-tree native libraries mapped into this process (proves the HIP kernels, not a fallback, ran)."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({os.path.basename(ln.split()[-1]) for ln in f if "libpdnn" in ln})
    except OSError:
        return []


def _plain_run(a):
    """Re-run this benchmark in a child process as the plain single-GPU step (no process group, no DDP wrapper);
    returns {value, ms_per_step} or an error note."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("PDNN_FORCE_PG", "PDNN_DDP_FORCE_COMM", "WORLD_SIZE",
                                                             "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    argv = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--steps", str(a.steps), "--warmup",
            str(a.warmup), "--model", a.model, "--bucket-mb", str(a.bucket_mb), "--graph", a.graph,
            "--plain"] + (["--batch", str(a.batch)] if a.batch else []) + (["--fp8"] if a.fp8 else [])
    try:
        r = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=900)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        rec = json.loads(line)
        return {"value": rec["value"], "ms_per_step": rec["ms_per_step"], "hipgraph": rec["config"]["hipgraph"],
                "note": "same model and step without the DDP wrapper / process group (no bucket hooks, no RCCL)"}
    except Exception as e:       # never lose the headline line over the second run
        return {"error": f"{type(e).__name__}: {e}"[:200]}


EXTRA_CONFIGS = (   # BASELINE.json configs 4 and 5, measured by the driver's one --gpus 1 command
    ("gpt2_small", ["--model", "gpt2_small"]),
    ("resnet152_bf16", ["--model", "resnet152"]),
    ("resnet152_fp8", ["--model", "resnet152", "--fp8"]),
)


def _child_run(a, extra, timeout=300):
    """This benchmark in a child process with ``extra`` arguments (the DDP code path at N = 1, no second plain run,
    no diagnostics); returns the child's headline fields or an error note."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    argv = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--steps", str(a.steps), "--warmup",
            str(a.warmup), "--no-plain-run", "--no-extra-configs", "--diag-steps", "0"] + extra
    t0 = time.perf_counter()
    try:
        r = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=timeout)
        rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        return {k: rec.get(k) for k in ("metric", "value", "unit", "ms_per_step", "dtype", "n1_point", "final_loss")} | {
            "config": {k: rec["config"].get(k) for k in ("model", "global_batch", "seq_len", "image_size", "bucket_mb")},
            "wall_s": round(time.perf_counter() - t0, 1)}
    except Exception as e:       # never lose the headline line over a secondary config
        return {"error": f"{type(e).__name__}: {e}"[:200], "wall_s": round(time.perf_counter() - t0, 1)}


def allreduce_probe(dev, world, sizes_mb=(32, 128), iters=10, warmup=3):
    """N > 1, after the timed region: bus bandwidth of back-to-back RCCL all-reduces (AVG, the DDP op) at the bucket
    sizes, fp32 and bf16 wire -- with 7 xGMI links per MI355X a ring is one link per hop, so busbw near one link's
    ~153 GB/s means RCCL is not spreading its channels over the links (tools/bench_allreduce.py, same method)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    from bench_allreduce import _one
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    out = []
    for dt in (torch.float32, torch.bfloat16):
        for mb in sizes_mb:
            r = _one("all_reduce", int(mb * 2 ** 20), dt, dev, world, iters, warmup, sync)
            out.append({"dtype": r["dtype"], "mib": mb, "us": r["us"], "busbw_GBps": r["busbw_GBps"]})
    return out


def comm_diagnostics(net, step, n):
    """{"bucket_mb", "fp32": {...}, "bf16": {...}}: per wire dtype, over ``n`` steps, the median per-bucket
    all-reduce device time (gradients ready -> reduced), when each bucket was ready / done relative to the first
    gradient hook, the exposed tail (last bucket done minus the backward's last kernel) and the BatchNorm-buffer
    broadcast; max over ranks."""
    import statistics
    out = {"bucket_mb": [round(v, 3) for v in net.bucket_sizes_mb()], "world": net.world}
    old = net.comm_dtype
    for name, dt in (("fp32", None), ("bf16", torch.bfloat16)):
        net.set_comm_dtype(dt)
        net.comm_timing = True
        net.comm_records()
        for i in range(n):
            step(i)
        torch.cuda.synchronize()
        net.comm_timing = False
        recs = net.comm_records()
        if not recs:
            out[name] = None
            continue
        med = lambda xs: statistics.median(xs)          # noqa: E731
        nb = len(recs[0]["bucket_ms"])
        r = {"bucket_allreduce_ms": [round(med([x["bucket_ms"][b] for x in recs]), 3) for b in range(nb)],
             "bucket_ready_ms": [round(med([x["bucket_ready_ms"][b] for x in recs]), 3) for b in range(nb)],
             "bucket_done_ms": [round(med([x["bucket_done_ms"][b] for x in recs]), 3) for b in range(nb)],
             "backward_end_ms": round(med([x["bwd_end_ms"] for x in recs]), 3),
             "exposed_tail_ms": round(med([x["tail_ms"] for x in recs]), 3),
             "bn_bcast_ms": (round(med([x["bn_bcast_ms"] for x in recs]), 3)
                             if recs[0]["bn_bcast_ms"] is not None else None)}
        if net.world > 1:       # max over ranks of the scalars (the slowest rank sets the step)
            v = torch.tensor([r["exposed_tail_ms"], r["bn_bcast_ms"] or 0.0, r["backward_end_ms"]], device=net.flat.grad.device)
            dist.all_reduce(v, op=dist.ReduceOp.MAX, group=net.pg)
            r["exposed_tail_ms"], r["bn_bcast_ms"], r["backward_end_ms"] = [round(x, 3) for x in v.tolist()]
        out[name] = r
    net.set_comm_dtype(old)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (256 images / 8 sequences)")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="DDP gradient bucket cap (default 32 MB; GPT-2 at N = 1 256 MB: there the all-reduce is a "
                         "no-op and every bucket collective only costs the compute stream a ~21 us stream-sync event, "
                         "gpurun_out/r5_44; 128 / 256 MB: 644.7k / 642.4k vs 646.9k / 647.0k tok/s, r6_28; ResNet-50 "
                         "32 / 64 / 128 MB equal there; at N > 1 the ddp.py cost model's 32 MB keeps every bucket but "
                         "the last under the backward)")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="at --gpus 1 (ResNet-50 headline), skip the child runs of BASELINE configs 4 and 5")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--fp8", action="store_true",
                    help="BASELINE config 5: ResNet 3x3 convs / GPT-2 forward linears on the fp8 MFMA kernels")
    ap.add_argument("--graph", default="auto", choices=["off", "on", "auto", "collectives"],
                    help="replay each step as one captured hipGraph (auto: single-GPU runs, not the side-stream ResNets)")
    ap.add_argument("--comm-bf16", action="store_true", help="DDP: all-reduce gradients in bf16 on the wire")
    ap.add_argument("--num-aggregate", type=int, default=0,
                    help="DDP k-of-n straggler mode with this k (control plane + host throttle on every step)")
    ap.add_argument("--plain", action="store_true",
                    help="one GPU without the DDP wrapper and process group (the second run of a --gpus 1 bench)")
    ap.add_argument("--no-ddp-rehearsal", "--no-plain-run", dest="no_plain_run", action="store_true",
                    help="at --gpus 1, skip the second measurement (the plain step)")
    ap.add_argument("--opt-overlap", action="store_true",
                    help="DDP path: apply the optimizer per bucket during the backward instead of after it")
    ap.add_argument("--diag-steps", type=int, default=5,
                    help="DDP path: extra steps after the timed region with per-bucket communication timing")
    ap.add_argument("--hang-timeout", type=float, default=90.0,
                    help="N > 1: hang watchdog (s without a completed step; the process-group timeout is 1.25x): "
                         "on a hang every rank prints one diagnostic JSON line and exits 75")
    a = ap.parse_args()
    if a.bucket_mb is None:
        n_world = int(os.environ.get("WORLD_SIZE", "1"))
        a.bucket_mb = 256.0 if a.model.lower().startswith("gpt2") and n_world == 1 else 32.0
    # stdout carries exactly the result line: libraries that print banners to fd 1 from C (RCCL's version block at
    # communicator init) are sent to stderr with everything else; the JSON lines go to the saved descriptor
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)

    def emit(rec):
        os.write(out_fd, (json.dumps(rec) + "\n").encode())

    from pytorch_distributed_nn_amd.parallel import runtime
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.optim import SGD, AdamW, flatten_module
    from pytorch_distributed_nn_amd.ops import functional as OF

    multi = int(os.environ.get("WORLD_SIZE", "1")) > 1
    if not multi and not a.plain:
        # BASELINE config 2 is "ResNet-50 bf16 DDP world_size=1": one GPU runs the same DDP code path as eight --
        # bucket hooks and an RCCL all-reduce of every bucket over a one-rank process group
        os.environ.setdefault("PDNN_FORCE_PG", "1")
        os.environ.setdefault("PDNN_DDP_FORCE_COMM", "1")
    # PDNN_BENCH_BACKEND: tests only (world 2 over gloo on a one-GPU box or on the CPU)
    backend = os.environ.get("PDNN_BENCH_BACKEND") or None
    env = runtime.init_process_group(backend=backend, device="cpu" if backend == "gloo" and not torch.cuda.is_available()
                                      else None, timeout_s=1.25 * a.hang_timeout if multi else 600.0)
    world = runtime.world_size()
    dev = runtime.device()
    on_gpu = dev.type == "cuda"

    def sync():
        if on_gpu:
            torch.cuda.synchronize()
    torch.manual_seed(1234 + env.rank)

    lm = a.model.lower().startswith("gpt2")
    # the reference's own configs: LeNet on MNIST, CIFAR-stem ResNets, batch 128 per worker, 10 classes
    # (pytorch_code/distributed_nn.py:42,58-63; model_ops/resnet.py:72,94)
    small = a.model.lower() == "lenet" or a.model.lower().endswith("_cifar")
    nc = 10 if small else 1000
    in_chw = (1, 28, 28) if a.model.lower() == "lenet" else (3, 32, 32) if small else (3, a.image_size, a.image_size)
    model = build_model(a.model, num_classes=nc).to(dev)
    if a.fp8:
        if lm:
            model.config.fp8 = True
        else:
            model.enable_fp8()
    if on_gpu and os.environ.get("PDNN_BENCH_COMM_WORLD"):
        # pricing runs only: make the kernels behave as one rank of a job this wide (the comm_cus reservation of the
        # persistent grids, csrc/kernels/tuning.h) while the process still runs a 1-rank group
        from pytorch_distributed_nn_amd.ops import kernels as _K
        _K.set_comm_world(int(os.environ["PDNN_BENCH_COMM_WORLD"]))
    use_ddp = world > 1 or os.environ.get("PDNN_DDP_FORCE_COMM") == "1"     # 1-GPU rehearsal of the DDP path
    if use_ddp:
        net = DistributedDataParallel(model, bucket_cap_mb=a.bucket_mb, num_aggregate=a.num_aggregate,
                                      comm_dtype=torch.bfloat16 if a.comm_bf16 else None)
    else:
        flatten_module(model)
        net = model
    if lm:
        opt = AdamW(model.parameters(), lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1)
        B, S = a.batch or 8, a.seq_len
        V = model.config.vocab_size
        toks = [torch.randint(0, min(50257, V), (B, S + 1), device=dev) for _ in range(2)]
        xs = [t[:, :-1].contiguous() for t in toks]
        ys = [t[:, 1:].contiguous() for t in toks]
    else:
        opt = SGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=5e-5)
        B, S = a.batch or (128 if small else 256), in_chw[-1]
        # bf16 images on the GPU; fp32 on the CPU (the gloo test rehearsal of the N > 1 path: torch's CPU convs)
        xs = [torch.randn(B, *in_chw, device=dev).to(torch.bfloat16 if on_gpu else torch.float32) for _ in range(2)]
        ys = [torch.randint(0, nc, (B,), device=dev) for _ in range(2)]

    # --opt-overlap: the DDP path applies each bucket's optimizer update as soon as the bucket is all-reduced,
    # beside the rest of the backward (DistributedDataParallel.overlap_optimizer).  Off by default: at N = 1 the
    # concurrent update slows the backward more than it hides (GPT-2 587k vs 593k tok/s, ResNet-50 11,575 vs
    # 11,616 img/s, gpurun_out/r5_29)
    opt_overlap = False
    if use_ddp and on_gpu and a.opt_overlap and isinstance(net, DistributedDataParallel):
        opt_overlap = net.overlap_optimizer(opt) is not None

    # auto: graphed on one GPU, except the ImageNet ResNets and GPT-2, whose weight gradients run on a side stream
    # concurrently with the data-gradient chain (ops/fused_resnet.py): eager launches overlap the two
    # streams (ResNet-50 8,635 vs 8,013 img/s serial), a replayed hipGraph ran the branches nearly serially
    # (8,160-8,196 img/s; gpurun_out/r2_32)
    from pytorch_distributed_nn_amd import tuning
    side_overlap = (not lm and not small and tuning.get("side_wgrad") == 1) or (
        lm and tuning.get("gpt2_side_wgrad") >= 1 and tuning.get("side_wgrad") == 1)
    use_graph = a.graph == "on" or (a.graph == "collectives") or (a.graph == "auto" and not use_ddp
                                                                   and not side_overlap)
    if use_graph:
        # whole step (fwd + bwd + optimizer [+ RCCL buckets if 'collectives']) replayed as one hipGraph
        from pytorch_distributed_nn_amd.utils.graphs import GraphedStep
        gstep = GraphedStep(net, opt, loss_fn=OF.cross_entropy, warmup=2,
                            forward=(lambda m, x, y: m(x, y)) if lm else None,
                            allow_collectives=a.graph == "collectives")

    def step(i):
        if use_graph:
            return gstep(xs[i % 2], ys[i % 2])
        opt.zero_grad()
        if lm:
            loss = net(xs[i % 2], ys[i % 2])
        else:
            loss = OF.cross_entropy(net(xs[i % 2]), ys[i % 2])
        if getattr(net, "kofn", None) is not None:
            net.backward(loss)
        else:
            loss.backward()
        opt.step()
        return loss

    # The side-stream ResNets run their compute stream at high priority (the side stream stays at the default,
    # lowest one): the wavefront dispatcher then fills the CUs with the critical-path data-gradient chain first
    # and the weight gradients take the gaps (+0.5% on ResNet-50, gpurun_out/r2_35).
    watchdog = None
    if world > 1:
        # a collective that never completes must not eat the driver's whole run: no step completed for
        # --hang-timeout seconds -> one JSON line per rank saying where it stood, then exit 75 (no re-exec)
        from pytorch_distributed_nn_amd.parallel.watchdog import EXIT_HANG, CommWatchdog

        def on_hang(rec):
            diag = {"metric": "hang", "error": f"no step completed for {rec['idle_s']} s", "rank": env.rank,
                    "world": world, "last_step_completed": rec["step"], "exit_code": EXIT_HANG,
                    "abort": rec.get("abort")}
            if isinstance(net, DistributedDataParallel):
                diag.update({("ddp_" + k if k == "step" else k): v for k, v in net.progress().items()})
            emit(diag)
        watchdog = CommWatchdog(timeout_s=a.hang_timeout, rank=env.rank, on_hang=on_hang).start()
    hang_at = int(os.environ.get("PDNN_BENCH_HANG_STEP", "-1"))       # tests: this step of the last rank never ends
    base_step = step

    def step(i):                                                        # noqa: F811
        if i == hang_at and env.rank == world - 1:
            while True:
                time.sleep(1)
        loss = base_step(i)
        if watchdog is not None:
            watchdog.beat(i)
        return loss

    ctx = contextlib.nullcontext()
    if side_overlap and dev.type == "cuda":
        main_stream = torch.cuda.Stream(device=dev, priority=-1)
        main_stream.wait_stream(torch.cuda.current_stream(dev))     # the data tensors were made on the default one
        ctx = torch.cuda.stream(main_stream)
    with ctx:
        for i in range(a.warmup):
            loss = step(i)
        runtime.barrier()
        sync()
        t0 = time.perf_counter()
        for i in range(a.steps):
            loss = step(a.warmup + i)
        runtime.barrier()
        sync()
    dt = time.perf_counter() - t0
    host_probe = None
    if os.environ.get("PDNN_BENCH_HOST_PROBE") and dev.type == "cuda":
        # diagnostics after the timed region: host enqueue time of one step started on an idle GPU vs the step's
        # wall time (a host time near the wall time = launch-bound); =2 also prints a cProfile of one step to stderr
        host_probe = []
        with ctx:
            for k in range(3):
                sync()
                h0 = time.perf_counter()
                step(a.warmup + a.steps + k)
                h1 = time.perf_counter()
                sync()
                host_probe.append({"host_ms": round((h1 - h0) * 1e3, 3), "wall_ms": round((time.perf_counter() - h0) * 1e3, 3)})
            if os.environ["PDNN_BENCH_HOST_PROBE"] == "2":
                import cProfile
                import pstats
                sync()
                pr = cProfile.Profile()
                pr.enable()
                step(a.warmup + a.steps + 3)
                pr.disable()
                sync()
                pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(40)
    comm = None
    if use_ddp and not use_graph and isinstance(net, DistributedDataParallel) and dev.type == "cuda":
        # after the timed region (it is not perturbed): a few more steps with device-event timing of every bucket
        # all-reduce, the exposed tail and the BN-buffer broadcast -- fp32 wire, then bf16 wire
        with ctx:
            comm = comm_diagnostics(net, step, a.diag_steps)
    if use_ddp and not on_gpu and isinstance(net, DistributedDataParallel):
        comm = {"bucket_mb": [round(v, 3) for v in net.bucket_sizes_mb()], "world": net.world, "fp32": None,
                "bf16": None, "note": "per-bucket device timing needs a GPU (CPU rehearsal)"}
    if world > 1 and isinstance(comm, dict):
        # bus bandwidth of the bucket-size collectives on this node (after the timed region)
        comm["allreduce_busbw"] = allreduce_probe(dev, world, iters=3 if not on_gpu else 10,
                                                  warmup=1 if not on_gpu else 3,
                                                  sizes_mb=(1, 4) if not on_gpu else (32, 128))
    if isinstance(comm, dict) and isinstance(net, DistributedDataParallel):
        comm["split_tied_embedding"] = net._tail is not None
    t = torch.tensor([dt], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    if watchdog is not None:
        watchdog.stop()
    ms = 1e3 * dt / a.steps
    value = B * world * a.steps / dt
    if getattr(net, "kofn", None) is not None:
        net.close()
    # At one GPU the plain step above is the N = 1 point of the scaling curve (the fastest 1-GPU
    # configuration); the same step through the DDP code path (bucket hooks, RCCL all-reduce of every bucket
    # over a one-rank process group) is measured in a child process and reported alongside, so a scaling
    # efficiency can be read against either.
    plain = None
    if world == 1 and use_ddp and not a.no_plain_run and env.rank == 0:
        plain = _plain_run(a)
    extra = None
    if (world == 1 and on_gpu and not a.plain and not a.no_extra_configs and a.model == "resnet50" and not a.fp8
            and env.rank == 0):
        extra = {name: _child_run(a, args) for name, args in EXTRA_CONFIGS}
    if lm and env.rank == 0:
        tok = value * S
        emit({
            "metric": "tokens/sec (whole node) GPT-2-small DDP",
            "value": round(tok, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp8(e4m3) fwd GEMMs + bf16" if a.fp8 else "bf16",
            "data": "synthetic (device-resident random token ids), random-init weights",
            "final_loss": round(float(loss.detach()), 4),
            "native_loaded": native_loaded(),
            "n1_point": "plain single-GPU step" if not use_ddp else
                        ("DDP path (1-rank process group: RCCL on a GPU)" if world == 1 else "DDP path"),
            "plain_step_1gpu": plain,
            "comm": comm,
            **({"host_probe": host_probe} if host_probe else {}),
            "model_tflops_per_gpu": round(tok / world * model.flops_per_token(S) / 1e12, 1),
            "config": {"model": f"{a.model} (12L/12H/768, vocab {V}, tied head)", "global_batch": B * world,
                       "per_gpu_batch": B, "seq_len": S, "parallelism": f"dp{world}",
                       "optimizer": "fused AdamW lr=6e-4 wd=0.1", "bucket_mb": a.bucket_mb, "hipgraph": use_graph,
                       "opt_overlap": opt_overlap},
        })
    elif env.rank == 0:
        emit({
            "metric": "samples/sec (whole node) ResNet-50 DDP" if a.model == "resnet50"
                      else f"samples/sec (whole node) {a.model} DDP",
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "vs_stock_pytorch_rocm": (round(value / (STOCK_PYTORCH_1GPU * world), 4)
                                      if a.model == "resnet50" and B == 256 and not a.fp8 else None),
            "dtype": "fp8 3x3 convs (e4m3 fwd / e5m2 dgrad) + bf16" if a.fp8 else "bf16" if on_gpu else "fp32 (CPU rehearsal)",
            "data": f"synthetic (device-resident random {in_chw[1]}x{in_chw[2]}x{in_chw[0]} images, random labels), "
                    "random-init weights",
            "final_loss": round(float(loss.detach()), 4),
            "native_loaded": native_loaded(),
            "n1_point": "plain single-GPU step" if not use_ddp else
                        ("DDP path (1-rank process group: RCCL on a GPU)" if world == 1 else "DDP path"),
            "plain_step_1gpu": plain,
            "extra_configs": extra,
            "comm": comm,
            **({"host_probe": host_probe} if host_probe else {}),
            "config": {"model": (f"{a.model} (reference layout, {in_chw[1]}x{in_chw[2]}, {nc} classes)" if small else
                                 f"{a.model} (ImageNet layout, {S}x{S}, {nc} classes)"), "global_batch": B * world,
                       "per_gpu_batch": B, "seq_len": None, "image_size": S, "parallelism": f"dp{world}",
                       "optimizer": "fused SGD momentum=0.9 wd=5e-5", "bucket_mb": a.bucket_mb, "hipgraph": use_graph,
                       "opt_overlap": opt_overlap},
        })
    runtime.destroy()


if __name__ == "__main__":
    main()
