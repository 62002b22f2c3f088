"""Native CLI (CPP-11/12) and run-report tooling (CPP-14, TF-09) on the CPU box."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def binary():
    from pytorch_distributed_nn_amd import _build
    return str(_build.build_tools())


def test_pdnn_mlp_single(binary):
    r = subprocess.run([binary, "single", "--iters", "5"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "final loss" in r.stdout


def test_pdnn_mlp_distributed_backup_workers(binary, tmp_path):
    out = str(tmp_path) + "/"
    r = subprocess.run([binary, "distributed", "--nprocs", "5", "--collect", "2", "--iters", "6", "--out", out],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    tl = [f for f in os.listdir(tmp_path) if f.startswith("timeline_out_")]
    tlo = [f for f in os.listdir(tmp_path) if f.startswith("time_loss_out_")]
    assert tl and tlo
    rep = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "report.py"), "timeline",
                          os.path.join(tmp_path, tl[0])], capture_output=True, text=True, timeout=60)
    assert rep.returncode == 0
    avg = float(rep.stdout.split("average gradients received per step")[1].split(",")[0])
    assert 2.0 <= avg <= 3.0          # >= n_to_collect per step; late (stale) arrivals are logged too


def test_pdnn_mlp_native_master_blocks_on_arrival_queue_and_drops_stale(binary, tmp_path):
    """the native master consumes a blocking arrival queue (no per-key polling); with 6
    workers and n_to_collect 2 the late gradients of closed steps are dropped by their step tag (the
    coordinator's stale path, sync_replicas_master_nn.h:85) and every gradient key is deleted."""
    out = str(tmp_path) + "/"
    r = subprocess.run([binary, "distributed", "--nprocs", "8", "--collect", "2", "--iters", "12", "--out", out],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    tl = [f for f in os.listdir(tmp_path) if f.startswith("timeline_out_")][0]
    summary = [ln for ln in open(os.path.join(tmp_path, tl)) if ln.startswith("# stale_dropped")][0].split()
    stale, leaked = int(summary[2]), int(summary[4])
    assert stale > 0 and leaked == 0, summary


def test_pdnn_mlp_fp64_matches_fp32(binary):
    """--fp64 runs the reference's double-precision arithmetic (cblas_dgemm, util.h:35-81); after 20 steps
    its loss agrees with the fp32 build to float rounding."""
    res = {}
    for flag in ([], ["--fp64"]):
        r = subprocess.run([binary, "single", "--iters", "20", *flag], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("final loss")][0]
        assert ("fp64" in line) == bool(flag)
        res[bool(flag)] = float(line.split()[2])
    assert abs(res[True] - res[False]) < 1e-3 * abs(res[False]), res


def test_report_percentiles(tmp_path):
    p = tmp_path / "m.jsonl"
    with open(p, "w") as f:
        for i in range(100):
            f.write(json.dumps({"step": i, "backward_ms": float(i)}) + "\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "report.py"), "percentiles", str(p)],
                       capture_output=True, text=True, timeout=60)
    rec = json.loads(r.stdout.strip())
    assert rec["n"] == 100 and abs(rec["p90"] - 89.1) < 1e-6


def test_cli_yaml_config_defaults(tmp_path):
    from pytorch_distributed_nn_amd.cli import parse_args
    import glob
    for f in glob.glob(os.path.join(ROOT, "configs", "**", "*.yaml"), recursive=True):
        parse_args(["--config", f])                                     # every shipped config parses
    a = parse_args(["--config", os.path.join(ROOT, "configs", "ps_mlp_backup_workers.yaml"), "--lr", "0.5"])
    assert a.network == "mlp_cpp" and a.n_to_collect == 2 and a.evaluator and a.lr == 0.5


def test_pmc_summary_flops_and_bytes(tmp_path):
    """tools/pmc_summary.py: 512 FLOPs per MFMA MOP, doubled FETCH_SIZE, per-dispatch timestamps."""
    hdr = "Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value,Start_Timestamp,End_Timestamp\n"
    with open(tmp_path / "q1_counters.csv", "w") as f:
        f.write(hdr)
        for c, v in (("SQ_INSTS_VALU_MFMA_MOPS_BF16", 1e6), ("SQ_LDS_BANK_CONFLICT", 1), ("SQ_LDS_IDX_ACTIVE", 4)):
            f.write(f"1,gemm,{c},{v},0,1000000\n")
    with open(tmp_path / "q2_counters.csv", "w") as f:
        f.write(hdr + "1,gemm,FETCH_SIZE,1000,0,1000000\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(tmp_path), "--steps", "1"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    row = [ln for ln in r.stdout.splitlines() if ln.endswith("gemm")][0].split()
    # 5.12e8 FLOP in 1 ms = 0.512 TFLOP/s; conflicts 1/4; read 2 x 1000 KiB in 1 ms = 2 GB/s
    assert float(row[2]) == pytest.approx(0.5, abs=0.05)
    assert float(row[4]) == pytest.approx(0.25)
    assert float(row[5]) == pytest.approx(2, abs=1)
