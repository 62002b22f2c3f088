"""``distnn-train`` command line (PT-01 pytorch_code/distributed_nn.py:36-102, PT-07 single_machine.py:28-55,
S4 tf flags).  All reference flag names and defaults are accepted verbatim:

  --batch-size 128  --test-batch-size 1000  --epochs 100  --lr 0.01  --momentum 0.5  --no-cuda  --seed 1
  --log-interval 10  --network LeNet  --dataset MNIST  --comm-type Bcast|Async  --num-aggregate 5

New:  --mode ddp|ps|single (default: ps when --comm-type is Bcast/Async and world > 1, i.e. the
reference's behaviour; ddp when --comm-type AllReduce), --comm-type AllReduce, --bucket-cap-mb,
--dtype bf16|fp32|fp8, --synthetic, --data-dir, --max-steps, --optimizer sgd|adam|adamw, --weight-decay,
--n-to-collect (backup workers), --interval-ms, --no-shortcircuit, --evaluator,
--inject-straggler RANK:MS[,RANK:MS], --straggler-mode (k-of-n inside DDP), --checkpoint-dir, --resume,
--trace FILE, --metrics FILE.

Launch:  torchrun --nproc-per-node N -m pytorch_distributed_nn_amd.cli ...   or   mpirun -n N python -m ...
"""
from __future__ import annotations

import argparse
import os

import torch


def add_fit_args(p: argparse.ArgumentParser):
    p.add_argument("--batch-size", type=int, default=128, metavar="N")
    p.add_argument("--test-batch-size", type=int, default=1000, metavar="N")
    p.add_argument("--epochs", type=int, default=100, metavar="N")
    p.add_argument("--lr", type=float, default=0.01, metavar="LR")
    p.add_argument("--momentum", type=float, default=0.5, metavar="M")
    p.add_argument("--no-cuda", action="store_true", default=False)
    p.add_argument("--seed", type=int, default=1, metavar="S")
    p.add_argument("--log-interval", type=int, default=10, metavar="N")
    p.add_argument("--network", type=str, default="LeNet", metavar="N")
    p.add_argument("--dataset", type=str, default="MNIST", metavar="N")
    p.add_argument("--comm-type", type=str, default="Bcast", choices=["Bcast", "Async", "AllReduce"])
    p.add_argument("--num-aggregate", type=int, default=5, metavar="N")
    # --- new
    p.add_argument("--mode", type=str, default=None, choices=["ddp", "ps", "single"])
    p.add_argument("--bucket-cap-mb", type=float, default=32.0)
    p.add_argument("--dtype", type=str, default="bf16", choices=["bf16", "fp32", "fp8"],
                   help="compute dtype on the GPU: bf16 (default), fp8 = BASELINE config 5 (the ResNet Bottlenecks' "
                        "3x3 convs / GPT-2's block linears on the fp8 MFMA kernels with delayed scaling, everything "
                        "else bf16; fp32 master weights in every case), fp32 = plain torch fp32 (no fused kernels)")
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--data-dir", type=str, default=None)
    p.add_argument("--max-steps", type=int, default=None)
    p.add_argument("--optimizer", type=str, default="sgd", choices=["sgd", "adam", "adamw"])
    p.add_argument("--weight-decay", type=float, default=0.0)
    # exponential staircase decay (TF trainer, distributed_TF/src/distributed_train.py:143-147):
    # lr = lr0 * factor ** floor(step / (steps_per_epoch * epochs_per_decay))
    p.add_argument("--lr-decay-factor", type=float, default=1.0)
    p.add_argument("--epochs-per-decay", type=float, default=0.0)
    p.add_argument("--num-workers", type=int, default=0, help="data-loader worker processes (0: a thread)")
    p.add_argument("--compute-times", action="store_true",
                   help="every rank appends per-step compute-time records to OUT_DIR/compute_times_rank<r>.jsonl "
                        "(TF timeout_manager.py:48-70 side channel; CDF/percentiles: tools/report.py cdf)")
    p.add_argument("--n-to-collect", type=int, default=0)
    p.add_argument("--interval-ms", type=float, default=0.0)
    p.add_argument("--no-shortcircuit", action="store_true")
    p.add_argument("--evaluator", action="store_true")
    p.add_argument("--eval-interval", type=int, default=10)
    p.add_argument("--inject-straggler", type=str, default="")
    p.add_argument("--straggler-mode", action="store_true")
    p.add_argument("--checkpoint-dir", type=str, default=None)
    p.add_argument("--resume", type=str, default=None, help="checkpoint path, or 'auto' (newest in --checkpoint-dir)")
    p.add_argument("--checkpoint-interval", type=int, default=0, help="rank 0 saves every N steps (0: per epoch)")
    p.add_argument("--watchdog-timeout", type=float, default=0.0,
                   help="seconds without a completed step before the rank aborts the communicator and exits "
                        "(code 75) for a torchrun --max-restarts restart; 0 = off")
    p.add_argument("--inject-hang", type=str, default="",
                   help="RANK:STEP - that rank stops making progress before step STEP on the FIRST attempt only "
                        "(fault injection for the watchdog + restart path; TORCHELASTIC_RESTART_COUNT == 0)")
    p.add_argument("--save-model-secs", type=float, default=0.0,
                   help="PS mode: the master checkpoints every N seconds of wall time into --checkpoint-dir, plus a "
                        "final save (TF Supervisor(save_model_secs) + chief save, distributed_train.py:215-223,346-350)")
    p.add_argument("--ps-workers", type=int, default=0,
                   help="PS mode: the number of gradient workers this launch must have (fails loudly otherwise; the "
                        "r-of-N sweeps need exactly N)")
    p.add_argument("--trace", type=str, default=None)
    p.add_argument("--graph", type=str, default="off", choices=["off", "on", "collectives"],
                   help="replay each training step as one captured hipGraph (utils/graphs.py); 'on' applies to "
                        "single-GPU runs, 'collectives' also captures the DDP all-reduces (every rank)")
    p.add_argument("--metrics", type=str, default=None)
    p.add_argument("--out-dir", type=str, default="outfiles")
    p.add_argument("--config", type=str, default=None,
                   help="YAML file of flag defaults (keys = flag names without '--'); explicit flags win")
    return p


def parse_args(argv=None):
    """Flags, with defaults optionally taken from a YAML experiment config (TF-11 cfg files).
    The YAML is read with ``yaml.safe_load``."""
    p = add_fit_args(argparse.ArgumentParser(description="pytorch_distributed_nn_amd trainer"))
    pre, _ = p.parse_known_args(argv)
    if pre.config:
        import yaml
        with open(pre.config) as f:
            cfg = yaml.safe_load(f) or {}
        known = {a.dest for a in p._actions}
        defaults = {}
        for k, v in cfg.items():
            dest = k.replace("-", "_")
            if dest not in known:
                raise SystemExit(f"{pre.config}: unknown option {k!r}")
            defaults[dest] = v
        p.set_defaults(**defaults)
    return p.parse_args(argv)


# flags each mode does not use: given explicitly (or by a YAML config) with a non-default value they are an
# error, never silently dropped (a PS sweep config that says "optimizer: adam" must run Adam or fail)
_PS_IGNORED = ("graph", "straggler_mode", "resume", "watchdog_timeout", "inject_hang", "trace", "metrics",
               "num_workers", "checkpoint_interval")
_COLLECTIVE_IGNORED = ("evaluator", "eval_interval", "no_shortcircuit", "save_model_secs", "ps_workers")
_STRAGGLER_ONLY = ("n_to_collect", "interval_ms", "num_aggregate")


def check_mode_flags(args, mode: str, world: int):
    """Raise SystemExit naming every flag the chosen mode would ignore."""
    base = vars(add_fit_args(argparse.ArgumentParser()).parse_args([]))
    given = {k for k, v in vars(args).items() if k in base and v != base[k] and k != "config"}
    bad = []
    if mode == "ps":
        bad += [k for k in _PS_IGNORED if k in given]
    else:
        bad += [k for k in _COLLECTIVE_IGNORED if k in given]
        if args.comm_type in ("Async",) and "comm_type" in given:
            bad.append("comm_type")
        if not (mode == "ddp" and args.straggler_mode and world > 1):
            bad += [k for k in _STRAGGLER_ONLY if k in given]
        if mode == "single" and "straggler_mode" in given:
            bad.append("straggler_mode")
    if bad:
        flags = ", ".join("--" + k.replace("_", "-") for k in sorted(set(bad)))
        raise SystemExit(f"--mode {mode} (world size {world}) does not use {flags}: remove them or pick the mode "
                         f"that implements them")


def parse_stragglers(s: str) -> dict:
    out = {}
    for part in filter(None, s.split(",")):
        r, ms = part.split(":")
        out[int(r)] = float(ms)
    return out


def main(argv=None):
    args = parse_args(argv)
    from .data.datasets import DataLoader, dataset_from_args
    from .models import build_model
    from .ops import functional as OF
    from .optim import SGD, Adam, AdamW, flatten_module
    from .parallel import runtime
    from .parallel.ddp import DistributedDataParallel
    from .trainer import Trainer

    torch.manual_seed(args.seed)
    env = runtime.init_process_group(device="cpu" if args.no_cuda else None)
    world, rank = runtime.world_size(), runtime.rank()
    dev = torch.device("cpu") if args.no_cuda or not torch.cuda.is_available() else runtime.device()
    mode = args.mode or ("single" if world == 1 else ("ddp" if args.comm_type == "AllReduce" else "ps"))
    check_mode_flags(args, mode, world)

    train_ds, test_ds = dataset_from_args(args.dataset, args.data_dir, args.synthetic, dev, args.batch_size,
                                          args.network)
    nc = 1000 if args.dataset.upper() == "IMAGENET" else 10
    model = build_model(args.network, nc).to(dev)
    if args.dtype == "fp8":
        if dev.type != "cuda":
            raise SystemExit("--dtype fp8 needs the GPU (the fp8 kernels are MFMA-only)")
        if hasattr(model, "enable_fp8"):
            model.enable_fp8()
        elif hasattr(getattr(model, "config", None), "fp8"):
            model.config.fp8 = True
        else:
            raise SystemExit(f"--dtype fp8: network {args.network} has no fp8 path (ResNet Bottlenecks, GPT-2)")
    xdt = torch.bfloat16 if (dev.type == "cuda" and args.dtype in ("bf16", "fp8")) else torch.float32

    def to_dev(batch):
        x, y = batch
        return x.to(dev, dtype=xdt, non_blocking=True), y.to(dev, non_blocking=True)

    if mode == "ps":
        from .parallel.ps import PSConfig, run_ps
        n_workers = world - (2 if args.evaluator else 1)
        if args.ps_workers and args.ps_workers != n_workers:
            raise SystemExit(f"--ps-workers {args.ps_workers}: this launch has {n_workers} workers (world {world} = "
                             f"master{' + evaluator' if args.evaluator else ''} + workers); launch "
                             f"{args.ps_workers + world - n_workers} processes")
        # TF staircase decay counts master updates: decay_steps = batches per epoch * epochs_per_decay / replicas
        # aggregated per update (distributed_train.py:138)
        agg = max(1, args.n_to_collect or n_workers)
        decay_steps = (max(1, int(len(train_ds) // args.batch_size * args.epochs_per_decay / agg))
                       if args.lr_decay_factor != 1.0 and args.epochs_per_decay > 0 else 0)
        cfg = PSConfig(compute_times=args.compute_times, log_compute_times=args.compute_times,
                       comm_type=args.comm_type if args.comm_type != "AllReduce" else "Bcast",
                       num_aggregate=args.num_aggregate if args.n_to_collect == 0 else 0,
                       n_to_collect=args.n_to_collect, shortcircuit=not args.no_shortcircuit,
                       interval_ms=args.interval_ms, evaluator=args.evaluator, eval_interval=args.eval_interval,
                       inject_straggler=parse_stragglers(args.inject_straggler), lr=args.lr, momentum=args.momentum,
                       weight_decay=args.weight_decay, optimizer=args.optimizer, lr_decay_factor=args.lr_decay_factor,
                       decay_steps=decay_steps, checkpoint_dir=args.checkpoint_dir or "",
                       save_model_secs=args.save_model_secs, max_steps=args.max_steps or 1000, out_dir=args.out_dir)
        wrank = max(0, rank - (2 if args.evaluator else 1))
        loader = DataLoader(train_ds, args.batch_size, "cpu", rank=wrank, world=max(1, n_workers))

        def batches():
            while True:
                yield to_dev(loader.next_batch())

        def evaluate(m):
            with torch.no_grad():
                x, y = test_ds.next_batch(min(args.test_batch_size, len(test_ds)))
                out = m(torch.as_tensor(x).to(dev, dtype=xdt))
                yt = torch.as_tensor(y).to(dev)
                return float(OF.cross_entropy(out, yt)), float((out.argmax(1) != yt).float().mean())

        out = run_ps(model, cfg, dev, loss_fn=OF.cross_entropy, batches=batches(), eval_fn=evaluate)
        if rank == 0:
            print(f"Master: finished {len(out)} steps; gradients used per step: {[r['count'] for r in out][-10:]}")
        runtime.destroy()
        return out

    net = model
    if mode == "ddp" and (world > 1 or os.environ.get("PDNN_DDP_FORCE_COMM") == "1"):
        # --straggler-mode: k-of-n kill (--num-aggregate k) or backup workers (--n-to-collect k) and/or a step
        # deadline (--interval-ms) in collective form (parallel/ddp.py)
        kofn = (args.n_to_collect or args.num_aggregate) if args.straggler_mode else 0
        net = DistributedDataParallel(model, bucket_cap_mb=args.bucket_cap_mb, straggler_mode=args.straggler_mode,
                                      num_aggregate=kofn, deadline_ms=args.interval_ms if args.straggler_mode else 0.0)
    else:
        flatten_module(model)
    params = model.parameters()
    if args.optimizer == "sgd":
        opt = SGD(params, lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay)
    elif args.optimizer == "adam":
        opt = Adam(params, lr=args.lr, weight_decay=args.weight_decay)
    else:
        opt = AdamW(params, lr=args.lr, weight_decay=args.weight_decay)
    if isinstance(net, DistributedDataParallel):
        net.attach_optimizer(opt)
    strag = parse_stragglers(args.inject_straggler)
    if rank in strag:
        import time as _t
        for p in model.parameters():
            p.register_post_accumulate_grad_hook(lambda _p, d=strag[rank] / 1e3: _t.sleep(d))

    if args.synthetic and dev.type == "cuda":
        # synthetic data lives in HBM like bench.py's: the input pipeline is not what is being measured
        from .data.datasets import DeviceDataLoader
        loader = DeviceDataLoader(train_ds, args.batch_size, dev, rank=rank, world=world, seed=args.seed, dtype=xdt)
    else:
        loader = DataLoader(train_ds, args.batch_size, "cpu", rank=rank, world=world, num_workers=args.num_workers,
                            seed=args.seed)

    hang_at = None
    if args.inject_hang and os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") == "0":
        hr, hs = (int(v) for v in args.inject_hang.split(":"))
        hang_at = hs if hr == rank else None

    class _DevLoader:
        def __iter__(self):
            n = 0
            while True:
                n += 1
                if hang_at is not None and n >= hang_at:      # a wedged rank: peers block in the all-reduce
                    import time as _t
                    while True:
                        _t.sleep(60)
                yield to_dev(loader.next_batch())

        def __len__(self):
            return len(loader)

        def skip(self, n):              # a resume fast-forward: the sampler only (Trainer.train)
            loader.skip(n)

    graph = {"off": False, "on": world == 1, "collectives": "collectives"}[args.graph]
    if strag:                      # per-step host sleeps in grad hooks cannot be replayed from a graph
        graph = False
    wd = None
    if args.watchdog_timeout > 0:
        from .parallel.watchdog import CommWatchdog
        wd = CommWatchdog(args.watchdog_timeout, out_dir=args.out_dir, rank=rank).start()
    lr_schedule = None
    if args.lr_decay_factor != 1.0 and args.epochs_per_decay > 0:
        decay_steps = max(1, int(len(loader) * args.epochs_per_decay))
        lr_schedule = lambda step, lr0=args.lr, f=args.lr_decay_factor: lr0 * f ** (step // decay_steps)  # noqa: E731
    tr = Trainer(net, opt, OF.cross_entropy, dev, rank, world, args.log_interval, args.metrics,
                 args.trace, args.checkpoint_dir, arch=args.network, printer=print if rank == 0 else (lambda *a: None),
                 graph=graph, checkpoint_interval=args.checkpoint_interval, watchdog=wd, lr_schedule=lr_schedule,
                 compute_log=(os.path.join(args.out_dir, f"compute_times_rank{rank}.jsonl")
                              if args.compute_times else None))
    if args.resume:
        ck = tr.resume(args.resume)
        if ck is not None and rank == 0:
            print(f"resumed from step {tr.step_no} (epoch {tr.epoch})")
    import contextlib
    ctx = contextlib.nullcontext()
    from . import tuning
    if dev.type == "cuda" and tuning.get("side_wgrad") == 1:
        # as bench.py: the fused ResNets' data-gradient chain runs on a high-priority stream, their weight
        # gradients on the default-priority side stream (ops/fused_resnet.py), so the dispatcher fills the CUs
        # with the critical path first
        main_stream = torch.cuda.Stream(device=dev, priority=-1)
        main_stream.wait_stream(torch.cuda.current_stream(dev))
        ctx = torch.cuda.stream(main_stream)
    with ctx:
        hist = tr.train(_DevLoader(), epochs=args.epochs, max_steps=args.max_steps, batch_size=args.batch_size,
                        dataset_size=len(train_ds))
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    test_loader = DataLoader(test_ds, min(args.test_batch_size, len(test_ds)), "cpu")

    class _TestLoader:
        def __iter__(self):
            while True:
                yield to_dev(test_loader.next_batch())

    if rank == 0:
        tr.evaluate(_TestLoader(), 1)
    if wd is not None:
        wd.stop()
    runtime.destroy()
    return hist


if __name__ == "__main__":
    main()
