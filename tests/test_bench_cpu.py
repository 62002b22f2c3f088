"""bench.py's N > 1 branch on the CPU over gloo (VERDICT r4 #3d): the driver's first 8-GPU run goes through code
that a one-GPU box cannot execute, so its host-side logic -- the world > 1 process group, the MAX-over-ranks
timing, the `comm` block and the hang watchdog -- runs here at world 2 (LeNet, fp32 CPU convs)."""
import json
import os
import subprocess
import sys

from dist_utils import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(nproc, args, env_extra, timeout):
    env = dict(os.environ, PDNN_BENCH_BACKEND="gloo", OMP_NUM_THREADS="1", **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--rdzv-backend", "c10d", "--rdzv-endpoint", f"127.0.0.1:{free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", str(nproc)] + args
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd="/tmp")


def _json_lines(out):
    recs = []
    for ln in out.splitlines():
        ln = ln.strip()
        if ln.startswith("{"):
            try:
                recs.append(json.loads(ln))
            except ValueError:
                pass
    return recs


def test_bench_world2_prints_one_line_with_comm_block():
    r = _torchrun(2, ["--model", "lenet", "--steps", "3", "--warmup", "1"], {}, 300)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout                      # rank 0 only
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 2 * rec["config"]["per_gpu_batch"]
    assert abs(rec["value"] - rec["config"]["global_batch"] * 1e3 / rec["ms_per_step"]) < 0.01 * rec["value"]
    assert rec["comm"]["world"] == 2 and len(rec["comm"]["bucket_mb"]) >= 1
    assert rec["n1_point"] == "DDP path"
    # at N > 1 the comm block carries the all-reduce bus-bandwidth probe (fp32 + bf16 wire)
    bw = rec["comm"]["allreduce_busbw"]
    assert {b["dtype"] for b in bw} == {"float32", "bfloat16"} and all(b["busbw_GBps"] > 0 for b in bw)
    assert rec["extra_configs"] is None          # the config-4/5 child runs belong to the 1-GPU command only


def test_bench_world2_gpt2_split_tied_embedding():
    """GPT-2 at N > 1: 32 MB bucket cap (256 MB only where the all-reduce is a no-op), the tied wte's LM-head part
    is bucket 0 and its embedding rows are gathered separately (comm.split_tied_embedding)."""
    r = _torchrun(2, ["--model", "gpt2_tiny", "--batch", "2", "--seq-len", "32", "--steps", "2", "--warmup", "1"],
                  {}, 300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["n_gpus"] == 2 and rec["config"]["bucket_mb"] == 32.0
    assert rec["comm"]["split_tied_embedding"] is True
    assert abs(rec["comm"]["bucket_mb"][0] - 512 * 128 * 4 / 2 ** 20) < 1e-6      # bucket 0 = the tied wte alone


def test_bench_world2_hang_prints_diagnostics_and_exits():
    """The last rank never finishes step 2: within the hang timeout every rank prints one JSON line saying
    where it stood (step, last bucket launched / completed) and the job exits non-zero -- instead of sitting
    in a collective until the driver's own limit."""
    r = _torchrun(2, ["--model", "lenet", "--steps", "4", "--warmup", "1", "--hang-timeout", "6"],
                  {"PDNN_BENCH_HANG_STEP": "2"}, 240)
    assert r.returncode != 0
    diags = [d for d in _json_lines(r.stdout) if d.get("metric") == "hang"]
    # the first rank whose watchdog fires exits 75 and torchrun then stops the others: at least one line
    assert diags, r.stdout + r.stderr[-2000:]
    for d in diags:
        assert d["world"] == 2 and d["exit_code"] == 75 and d["last_step_completed"] == 1
        assert "last_bucket_launched" in d and "last_bucket_completed" in d and "buckets_in_flight" in d
        if d["rank"] == 0:        # waiting inside step 2's (the third DDP step's) gradient reduction
            assert d["ddp_step"] == 3 and d["in_backward"]
        else:                     # the wedged rank never started step 2's backward
            assert d["ddp_step"] == 2 and not d["in_backward"]
