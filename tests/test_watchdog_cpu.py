"""Hang detection + restart-from-checkpoint (parallel/watchdog.py).  The reference
has no recovery: a wedged rank stalls every peer forever (pytorch_code/sync_replicas_master_nn.py:148-150)."""
import json
import os
import subprocess
import sys
import time

from dist_utils import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_watchdog_fires_without_heartbeat_and_not_with_it(tmp_path):
    from pytorch_distributed_nn_amd.parallel.watchdog import CommWatchdog
    fired = []
    wd = CommWatchdog(0.4, out_dir=str(tmp_path), rank=3, exit_on_hang=False, on_hang=fired.append,
                      poll_s=0.05).start()
    for i in range(12):                 # beating every 0.1 s: never idle for 0.4 s
        time.sleep(0.1)
        wd.beat(i)
    assert not fired
    time.sleep(0.8)                     # stop beating: the step "hangs"
    wd.stop()
    assert len(fired) == 1 and fired[0]["rank"] == 3 and fired[0]["step"] == 11
    rec = json.load(open(tmp_path / "hang_rank3.json"))
    assert rec["idle_s"] >= 0.4 and "MainThread" not in rec["abort"] and rec["stacks"]


def test_latest_checkpoint(tmp_path):
    from pytorch_distributed_nn_amd.parallel.watchdog import latest_checkpoint
    assert latest_checkpoint(str(tmp_path)) is None
    for i, n in enumerate(["checkpoint_step2.pt", "checkpoint_step10.pt", "checkpoint_step4.pt"]):
        p = tmp_path / n
        p.write_bytes(b"x")
        os.utime(p, (1000 + i, 1000 + i))
    assert latest_checkpoint(str(tmp_path)).endswith("checkpoint_step4.pt")      # newest written wins


def test_hang_restart_resume_end_to_end(tmp_path):
    """2 ranks under torchrun (gloo): rank 1 wedges before its 5th step on the first attempt; the
    watchdogs end both ranks with code 75, torchrun restarts the group, it resumes from the newest
    checkpoint and finishes all 10 steps."""
    ck, out = tmp_path / "ck", tmp_path / "out"
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--rdzv-backend", "c10d", "--rdzv-endpoint", f"127.0.0.1:{free_port()}", "--max-restarts", "1",
           "-m", "pytorch_distributed_nn_amd.cli", "--no-cuda", "--comm-type", "AllReduce", "--network", "LeNet",
           "--synthetic", "--max-steps", "10", "--epochs", "20", "--log-interval", "2", "--checkpoint-dir", str(ck),
           "--checkpoint-interval", "2", "--resume", "auto", "--watchdog-timeout", "4", "--inject-hang", "1:5",
           "--out-dir", str(out)]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=240)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-4000:]
    assert "exiting with 75" in log and "resumed from step 4" in log, log[-4000:]
    assert list(out.glob("hang_rank*.json"))          # whichever rank noticed first
    assert (ck / "checkpoint_step10.pt").exists()
