"""Multi-node cluster tooling for MI355X nodes.

The reference provisions AWS EC2 spot instances and drives them over ssh (tools/pytorch_ec2.py:176-256
launch / wait, :656-819 get_hosts -> ``hosts`` / ``hosts_alias`` / ``hosts_address`` files, :821-878
kill_python / kill_all_python / run_command, :880-900 NFS setup; distributed_TF/tools/tf_ec2.py:504-535
parallel ssh with PS_HOSTS / TASK_ID / JOB_NAME placeholder substitution, :605-694 result download with a
vendored scp client).  Cloud provisioning has no counterpart here (MI355X nodes are allocated by the site
scheduler, e.g. SLURM), but everything after "the machines exist" does:

=========  ==========================================================================================
verb       what it does
=========  ==========================================================================================
hosts      write ``hosts`` (addresses), ``hosts_alias`` (``addr alias``) and ``hosts_address`` files from
           ``--hosts h1,h2`` / a cluster YAML / ``SLURM_JOB_NODELIST`` (TL-01 get_hosts, TL-05 files)
launch     start one ``torch.distributed.run`` per node (``--nnodes N --node-rank i --nproc-per-node G``,
           master = first node) in the background, one PID file per node (TL-01 launch, TF-08 run_tf)
run        run a shell command on every node in parallel and collect the outputs (TL-04 pdsh fan-out,
           TL-01 run_command); ``{NODE_RANK}`` / ``{HOST}`` / ``{MASTER}`` / ``{NNODES}`` placeholders are
           substituted per node like the reference's PS_HOSTS / TASK_ID templates (tf_ec2.py:476-502)
status     is each node's launched job still alive (its recorded PID)
kill       stop each node's launched job by its recorded process group — never by name pattern (the
           reference's kill_all_python kills every python on the machine)
fetch      copy a remote directory (logs, metrics, checkpoints) back per node (TF-10 scp, TF-08 download)
=========  ==========================================================================================

Transport is ``ssh``/``scp`` (BatchMode, optional key/user), or ``local`` (commands run on this machine,
every "node" a local process): the single-node MI355X pool and the CPU tests use that.

    python -m pytorch_distributed_nn_amd.cluster hosts  --hosts 10.0.0.1,10.0.0.2 --out cluster/
    python -m pytorch_distributed_nn_amd.cluster launch --hosts 10.0.0.1,10.0.0.2 --gpus 8 \\
        --repo /shared/repo --log-dir /shared/runs/r1 -- bench.py --steps 50
    python -m pytorch_distributed_nn_amd.cluster kill   --hosts 10.0.0.1,10.0.0.2 --log-dir /shared/runs/r1
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import re
import shlex
import subprocess
import sys
from dataclasses import dataclass, field


# ------------------------------------------------------------------------------------------------ hosts
def expand_nodelist(spec: str) -> list[str]:
    """SLURM-style ``node[01-03,07],login`` -> [node01, node02, node03, node07, login]."""
    out, i, parts, depth, cur = [], 0, [], 0, ""
    for ch in spec:                       # split on commas outside brackets
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
            continue
        depth += ch == "["
        depth -= ch == "]"
        cur += ch
    if cur:
        parts.append(cur)
    for p in parts:
        m = re.fullmatch(r"(.*)\[([^\]]+)\](.*)", p)
        if not m:
            out.append(p)
            continue
        pre, body, post = m.groups()
        for rng in body.split(","):
            if "-" in rng:
                a, b = rng.split("-")
                for n in range(int(a), int(b) + 1):
                    out.append(f"{pre}{str(n).zfill(len(a))}{post}")
            else:
                out.append(f"{pre}{rng}{post}")
        i += 1
    return out


@dataclass
class Cluster:
    hosts: list[str]
    aliases: list[str] = field(default_factory=list)
    user: str | None = None
    key: str | None = None
    transport: str = "ssh"
    repo: str = "."
    python: str = "python"
    gpus: int = 8
    port: int = 29500

    def __post_init__(self):
        if not self.hosts:
            raise ValueError("cluster: no hosts")
        if not self.aliases:
            self.aliases = [f"mi355x-node{i}" for i in range(len(self.hosts))]

    @property
    def master(self):
        return self.hosts[0]

    # -------------------------------------------------------------------------------------- transport
    def _ssh_target(self, host):
        return f"{self.user}@{host}" if self.user else host

    def remote_argv(self, host: str, cmd: str) -> list[str]:
        if self.transport == "local":
            return ["bash", "-c", cmd]
        argv = ["ssh", "-o", "BatchMode=yes", "-o", "StrictHostKeyChecking=accept-new"]
        if self.key:
            argv += ["-i", self.key]
        return argv + [self._ssh_target(host), cmd]

    def copy_argv(self, host: str, remote: str, local: str) -> list[str]:
        if self.transport == "local":
            return ["bash", "-c", f"mkdir -p {shlex.quote(local)} && cp -r {shlex.quote(remote)}/. {shlex.quote(local)}/"]
        argv = ["scp", "-r", "-o", "BatchMode=yes"]
        if self.key:
            argv += ["-i", self.key]
        return argv + [f"{self._ssh_target(host)}:{remote}/.", local]

    def subst(self, cmd: str, rank: int) -> str:
        return (cmd.replace("{NODE_RANK}", str(rank)).replace("{HOST}", self.hosts[rank])
                .replace("{MASTER}", self.master).replace("{NNODES}", str(len(self.hosts))))

    def fan_out(self, argvs: list[list[str]], timeout: float | None = 600) -> list[subprocess.CompletedProcess]:
        with cf.ThreadPoolExecutor(max_workers=min(32, len(argvs))) as ex:
            futs = [ex.submit(subprocess.run, a, capture_output=True, text=True, timeout=timeout) for a in argvs]
            return [f.result() for f in futs]

    # ------------------------------------------------------------------------------------------- verbs
    def write_hosts(self, out_dir: str):
        """TL-01 get_hosts: ``hosts`` (one address per line), ``hosts_alias`` (``addr alias``), and
        ``hosts_address`` (the ``addr:port`` list the launch line uses)."""
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, "hosts"), "w") as f:
            f.write("".join(h + "\n" for h in self.hosts))
        with open(os.path.join(out_dir, "hosts_alias"), "w") as f:
            f.write("".join(f"{h} {a}\n" for h, a in zip(self.hosts, self.aliases)))
        with open(os.path.join(out_dir, "hosts_address"), "w") as f:
            f.write(",".join(f"{h}:{self.port}" for h in self.hosts) + "\n")
        return [os.path.join(out_dir, n) for n in ("hosts", "hosts_alias", "hosts_address")]

    def launch_cmds(self, script_args: list[str], log_dir: str, env: dict | None = None) -> list[str]:
        nn = len(self.hosts)
        envs = " ".join(f"{k}={shlex.quote(str(v))}" for k, v in (env or {}).items())
        cmds = []
        for i in range(nn):
            run = (f"{self.python} -m torch.distributed.run --nnodes {nn} --node-rank {i} "
                   f"--nproc-per-node {self.gpus} --master-addr {self.master} --master-port {self.port} "
                   + " ".join(shlex.quote(a) for a in script_args))
            log = f"{log_dir}/node{i}.log"
            pid = f"{log_dir}/node{i}.pid"
            # braces: only the launcher goes to the background (so $! is its PID, and the ssh/bash session
            # returns at once); setsid makes it a process-group leader that `kill` can signal as a whole
            cmds.append(f"mkdir -p {shlex.quote(log_dir)} && cd {shlex.quote(self.repo)} && "
                        f"{{ {envs + ' ' if envs else ''}setsid nohup {run} > {shlex.quote(log)} 2>&1 < /dev/null & "
                        f"echo $! > {shlex.quote(pid)}; }}")
        return cmds

    def launch(self, script_args, log_dir, env=None):
        return self.fan_out([self.remote_argv(h, c) for h, c in zip(self.hosts, self.launch_cmds(script_args, log_dir, env))])

    def run(self, cmd: str, timeout=600):
        return self.fan_out([self.remote_argv(h, self.subst(cmd, i)) for i, h in enumerate(self.hosts)], timeout)

    def status(self, log_dir: str) -> list[bool]:
        cmd = "kill -0 $(cat {d}/node{{NODE_RANK}}.pid) 2>/dev/null && echo alive || echo dead".format(d=log_dir)
        return [r.stdout.strip().endswith("alive") for r in self.run(cmd)]

    def kill(self, log_dir: str, sig: str = "TERM"):
        # setsid made the launcher the leader of its own process group: signal exactly that group
        cmd = (f"p=$(cat {log_dir}/node{{NODE_RANK}}.pid 2>/dev/null) && kill -{sig} -- -$p 2>/dev/null; "
               f"true")
        return self.run(cmd)

    def fetch(self, remote_dir: str, local_dir: str):
        return self.fan_out([self.copy_argv(h, remote_dir, os.path.join(local_dir, a))
                             for h, a in zip(self.hosts, self.aliases)])


def cluster_from_args(a) -> Cluster:
    hosts, aliases = [], []
    if a.config:
        import yaml
        with open(a.config) as f:
            cfg = yaml.safe_load(f) or {}
        for n in cfg.get("nodes", []):
            hosts.append(n["host"] if isinstance(n, dict) else str(n))
            if isinstance(n, dict) and n.get("alias"):
                aliases.append(n["alias"])
        for k in ("user", "key", "transport", "repo", "python", "gpus", "port"):
            if k in cfg and getattr(a, k, None) in (None, ""):
                setattr(a, k, cfg[k])
    if a.hosts:
        hosts = expand_nodelist(a.hosts)
    elif not hosts and os.environ.get("SLURM_JOB_NODELIST"):
        hosts = expand_nodelist(os.environ["SLURM_JOB_NODELIST"])
    return Cluster(hosts=hosts, aliases=aliases if len(aliases) == len(hosts) else [], user=a.user, key=a.key,
                   transport=a.transport or "ssh", repo=a.repo or ".", python=a.python or "python",
                   gpus=int(a.gpus or 8), port=int(a.port or 29500))


def main(argv=None):
    ap = argparse.ArgumentParser(description="MI355X multi-node tooling (hosts / launch / run / status / kill / fetch)")
    ap.add_argument("verb", choices=["hosts", "launch", "run", "status", "kill", "fetch"])
    ap.add_argument("--hosts", default=None, help="h1,h2 or a SLURM nodelist (default: $SLURM_JOB_NODELIST)")
    ap.add_argument("--config", default=None, help="cluster YAML: nodes: [{host, alias}], user, key, repo, gpus, port")
    ap.add_argument("--user", default=None)
    ap.add_argument("--key", default=None)
    ap.add_argument("--transport", default=None, choices=["ssh", "local"])
    ap.add_argument("--repo", default=None)
    ap.add_argument("--python", default=None)
    ap.add_argument("--gpus", default=None)
    ap.add_argument("--port", default=None)
    ap.add_argument("--out", default="cluster", help="hosts: output directory")
    ap.add_argument("--log-dir", default="runs/latest")
    ap.add_argument("--cmd", default=None, help="run: shell command ({NODE_RANK} {HOST} {MASTER} {NNODES})")
    ap.add_argument("--remote", default=None, help="fetch: remote directory (default: --log-dir)")
    ap.add_argument("--dry-run", action="store_true")
    argv = list(sys.argv[1:] if argv is None else argv)
    script = []
    if "--" in argv:                                  # launch: everything after -- is the training command
        k = argv.index("--")
        argv, script = argv[:k], argv[k + 1:]
    a = ap.parse_args(argv)
    c = cluster_from_args(a)
    if a.verb == "hosts":
        for p in c.write_hosts(a.out):
            print(p)
        return 0
    if a.verb == "launch":
        if not script:
            ap.error("launch: give the training script after --")
        if a.dry_run:
            for h, cmd in zip(c.hosts, c.launch_cmds(script, a.log_dir)):
                print(" ".join(shlex.quote(x) for x in c.remote_argv(h, cmd)))
            return 0
        res = c.launch(script, a.log_dir)
    elif a.verb == "run":
        res = c.run(a.cmd or "hostname")
    elif a.verb == "status":
        for h, alive in zip(c.hosts, c.status(a.log_dir)):
            print(f"{h}: {'alive' if alive else 'dead'}")
        return 0
    elif a.verb == "kill":
        res = c.kill(a.log_dir)
    else:
        res = c.fetch(a.remote or a.log_dir, a.out)
    rc = 0
    for h, r in zip(c.hosts, res):
        print(f"[{h}] rc={r.returncode} {r.stdout.strip()} {r.stderr.strip()}".rstrip())
        rc = rc or r.returncode
    return rc


if __name__ == "__main__":
    sys.exit(main())
