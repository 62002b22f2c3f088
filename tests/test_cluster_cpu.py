"""Multi-node tooling (pytorch_distributed_nn_amd/cluster.py):
hosts files, per-node torchrun launch lines, placeholder fan-out, PID-file status/kill and result fetch,
exercised with the local transport (every "node" a local process)."""
import os
import time

from pytorch_distributed_nn_amd.cluster import Cluster, expand_nodelist, main


def test_expand_nodelist():
    assert expand_nodelist("gpu[01-03,07],login") == ["gpu01", "gpu02", "gpu03", "gpu07", "login"]
    assert expand_nodelist("a,b") == ["a", "b"]


def test_hosts_files(tmp_path):
    c = Cluster(hosts=["10.0.0.1", "10.0.0.2"], port=29600)
    c.write_hosts(str(tmp_path))
    assert (tmp_path / "hosts").read_text() == "10.0.0.1\n10.0.0.2\n"
    assert (tmp_path / "hosts_alias").read_text() == "10.0.0.1 mi355x-node0\n10.0.0.2 mi355x-node1\n"
    assert (tmp_path / "hosts_address").read_text() == "10.0.0.1:29600,10.0.0.2:29600\n"


def test_launch_lines_and_ssh_argv():
    c = Cluster(hosts=["n0", "n1", "n2"], user="me", key="/k", repo="/r", gpus=8, port=29500)
    cmds = c.launch_cmds(["bench.py", "--steps", "5"], "/runs/x")
    assert len(cmds) == 3
    for i, cmd in enumerate(cmds):
        assert f"--nnodes 3 --node-rank {i} --nproc-per-node 8 --master-addr n0 --master-port 29500" in cmd
        assert "bench.py --steps 5" in cmd and f"/runs/x/node{i}.pid" in cmd and "cd /r" in cmd
    argv = c.remote_argv("n1", "hostname")
    assert argv[0] == "ssh" and "-i" in argv and "me@n1" in argv and argv[-1] == "hostname"
    assert c.subst("echo {NODE_RANK} {HOST} {MASTER} {NNODES}", 2) == "echo 2 n2 n0 3"


def test_local_transport_run_launch_status_kill_fetch(tmp_path):
    c = Cluster(hosts=["127.0.0.1", "localhost"], transport="local", repo=str(tmp_path), python="python")
    outs = c.run("echo rank={NODE_RANK} of {NNODES}")
    assert [r.stdout.strip() for r in outs] == ["rank=0 of 2", "rank=1 of 2"]
    # a long-running "job" per node instead of torchrun: launch_cmds' structure with a sleeper
    logs = tmp_path / "runs"
    cmds = [f"mkdir -p {logs} && {{ setsid nohup sleep 60 > {logs}/node{i}.log 2>&1 < /dev/null & "
            f"echo $! > {logs}/node{i}.pid; }}" for i in range(2)]
    c.fan_out([c.remote_argv(h, cmd) for h, cmd in zip(c.hosts, cmds)])
    time.sleep(0.3)
    assert c.status(str(logs)) == [True, True]
    c.kill(str(logs))
    for _ in range(50):
        if c.status(str(logs)) == [False, False]:
            break
        time.sleep(0.1)
    assert c.status(str(logs)) == [False, False]
    (logs / "metrics.jsonl").write_text("{}\n")
    c.fetch(str(logs), str(tmp_path / "fetched"))
    for a in c.aliases:
        assert (tmp_path / "fetched" / a / "metrics.jsonl").exists()


def test_cli_hosts_and_dry_run(tmp_path, capsys):
    assert main(["hosts", "--hosts", "h[1-2]", "--out", str(tmp_path)]) == 0
    assert (tmp_path / "hosts").read_text() == "h1\nh2\n"
    capsys.readouterr()
    assert main(["launch", "--hosts", "h1,h2", "--dry-run", "--gpus", "8", "--", "bench.py", "--gpus", "16"]) == 0
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 2 and "--node-rank 1" in out[1] and out[0].startswith("ssh ")
