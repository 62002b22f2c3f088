"""Wall-clock throughput of the north-star entrypoint (``cli.py``'s Trainer.train) against bench.py.

python tools/cli_vs_bench.py METRICS.jsonl BENCH.json [--batch 256]

METRICS.jsonl is ``cli.py --metrics``: every log-interval record carries ``wall_s``, taken after that step
completed on the device.  The CLI throughput is (steps between the first and last logged record) x batch /
elapsed wall time -- the same whole-step, host-included measure as bench.py's timed loop.  Prints one JSON
line with both numbers and their ratio."""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("metrics")
    ap.add_argument("bench")
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    pts = [json.loads(ln) for ln in open(a.metrics) if ln.strip()]
    pts = [(r["step"], r["wall_s"]) for r in pts if r.get("wall_s")]
    (s0, t0), (s1, t1) = pts[0], pts[-1]
    cli = (s1 - s0) * a.batch / (t1 - t0)
    b = json.loads([ln for ln in open(a.bench) if ln.startswith("{")][-1])
    ddp = b["value"]                                            # bench's headline: the DDP path at every N
    plain = (b.get("plain_step_1gpu") or {}).get("value")
    print(json.dumps({"cli_samples_per_s": round(cli, 1), "cli_steps": s1 - s0, "bench_ddp_path": ddp,
                      "bench_plain": plain, "cli_vs_bench_ddp": round(cli / ddp, 4),
                      "cli_vs_bench_plain": round(cli / plain, 4) if plain else None}))


if __name__ == "__main__":
    main()
