"""Multi-node launcher: hostfile -> one agent per node -> one process per GPU slot.

Reference behaviour: ``deepspeed --hostfile=./hostfile --master_addr=$MASTER_ADDR
zero_dp_training.py --stage=2 ...`` (scripts/launch-multinode.sh:5).  The DeepSpeed runner parses
``host slots=N`` lines, fans out over pdsh, and each node's ``deepspeed.launcher.launch`` starts one
process per slot with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set and
``--local_rank=i`` appended.  Empty ``--master_addr`` falls back to the first host.

This module supplies the same contract without pdsh or MPI:

* ``parse_hostfile`` / ``select_hosts`` -- DeepSpeed hostfile syntax (``#`` comments, ``slots=``),
  ``--include`` / ``--exclude`` filters (``host1:0,1@host2``), ``--num_nodes`` / ``--num_gpus``.
* ``NodeAgent`` -- runs on each node: starts ``slots`` children in their own process groups with the
  torchrun env contract plus ``LOCAL_WORLD_SIZE`` / ``NODE_RANK`` and ``HIP_VISIBLE_DEVICES`` left
  untouched (one process per MI355X, selected by LOCAL_RANK inside ``comm.init``).  The first child
  that exits non-zero terminates its siblings (fail-fast) and becomes the exit code.
* the runner -- single-host hostfiles (or none) run the agent in-process; otherwise one ``ssh`` per
  node starts ``python -m ...launch.multinode --node-rank i`` there, forwarding the RCCL/HSA/HIP
  environment (and a ``.dtd_env`` file, like DeepSpeed's ``.deepspeed_env``).

Quirks of the reference fixed deliberately: the master address is resolved on
the launching host (never expands to empty on the remote side), and unknown script flags are passed
through verbatim instead of silently swallowed.
"""
from __future__ import annotations

import argparse
import os
import shlex
import signal
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field

FORWARD_ENV_PREFIXES = ("NCCL_", "RCCL_", "HSA_", "HIP_", "ROCR_", "TORCH_", "PYTORCH_", "OMP_", "MIOPEN_",
                        "HIPBLASLT_", "ROCBLAS_", "DTD_")
FORWARD_ENV_NAMES = ("PYTHONPATH", "PATH", "LD_LIBRARY_PATH")
ENV_FILE = ".dtd_env"
LOCAL_NAMES = {"localhost", "127.0.0.1", "::1"}


@dataclass
class Host:
    name: str
    slots: int
    devices: list[int] = field(default_factory=list)   # local device ids (default 0..slots-1)

    def __post_init__(self):
        if not self.devices:
            self.devices = list(range(self.slots))


def parse_hostfile(text: str) -> list[Host]:
    """``hostname slots=N`` per line; blank lines and ``#`` comments ignored; duplicate hosts rejected."""
    hosts: list[Host] = []
    seen = set()
    for ln, raw in enumerate(text.splitlines(), 1):
        line = raw.split("#", 1)[0].strip()
        if not line:
            continue
        parts = line.split()
        name, slots = parts[0], None
        for tok in parts[1:]:
            if tok.startswith("slots="):
                slots = int(tok.split("=", 1)[1])
            else:
                raise ValueError(f"hostfile line {ln}: unexpected token {tok!r}")
        if slots is None or slots <= 0:
            raise ValueError(f"hostfile line {ln}: missing or invalid slots= for {name!r}")
        if name in seen:
            raise ValueError(f"hostfile line {ln}: duplicate host {name!r}")
        seen.add(name)
        hosts.append(Host(name, slots))
    if not hosts:
        raise ValueError("hostfile lists no hosts")
    return hosts


def _parse_filter(spec: str) -> dict[str, list[int] | None]:
    out: dict[str, list[int] | None] = {}
    for item in filter(None, spec.split("@")):
        if ":" in item:
            name, devs = item.split(":", 1)
            out[name] = [int(d) for d in devs.split(",") if d != ""]
        else:
            out[item] = None
    return out


def select_hosts(hosts: list[Host], include: str = "", exclude: str = "", num_nodes: int = -1,
                 num_gpus: int = -1) -> list[Host]:
    """Apply DeepSpeed-style ``--include`` / ``--exclude`` / ``--num_nodes`` / ``--num_gpus`` filters."""
    if include and exclude:
        raise ValueError("--include and --exclude are mutually exclusive")
    res = [Host(h.name, h.slots, list(h.devices)) for h in hosts]
    names = {h.name for h in res}
    if include:
        inc = _parse_filter(include)
        for n in inc:
            if n not in names:
                raise ValueError(f"--include names unknown host {n!r}")
        res = [h for h in res if h.name in inc]
        for h in res:
            if inc[h.name] is not None:
                bad = [d for d in inc[h.name] if d not in h.devices]
                if bad:
                    raise ValueError(f"--include: {h.name} has no slot(s) {bad}")
                h.devices = list(inc[h.name])
    if exclude:
        exc = _parse_filter(exclude)
        for n in exc:
            if n not in names:
                raise ValueError(f"--exclude names unknown host {n!r}")
        kept = []
        for h in res:
            if h.name in exc:
                if exc[h.name] is None:
                    continue
                h.devices = [d for d in h.devices if d not in exc[h.name]]
                if not h.devices:
                    continue
            kept.append(h)
        res = kept
    if num_nodes > 0:
        res = res[:num_nodes]
    if num_gpus > 0:
        for h in res:
            h.devices = h.devices[:num_gpus]
    for h in res:
        h.slots = len(h.devices)
    if not res:
        raise ValueError("no hosts left after filtering")
    return res


@dataclass(frozen=True)
class RankInfo:
    host: str
    node_rank: int
    local_rank: int
    rank: int
    device: int


def rank_table(hosts: list[Host]) -> list[RankInfo]:
    """Global ranks are assigned node-major (node 0's slots first), as torchrun and DeepSpeed do."""
    out, r = [], 0
    for n, h in enumerate(hosts):
        for lr, dev in enumerate(h.devices):
            out.append(RankInfo(h.name, n, lr, r, dev))
            r += 1
    return out


def is_local(name: str) -> bool:
    return name in LOCAL_NAMES or name in (socket.gethostname(), socket.getfqdn())


def forwarded_env(environ: dict[str, str] | None = None, env_file: str | None = ENV_FILE) -> dict[str, str]:
    """The environment a remote node must see: RCCL/HSA/HIP/torch knobs plus ``.dtd_env`` lines."""
    environ = dict(os.environ if environ is None else environ)
    out = {k: v for k, v in environ.items() if k.startswith(FORWARD_ENV_PREFIXES) or k in FORWARD_ENV_NAMES}
    # dmabuf IPC is the only peer-memory path the MI355X host driver supports (RCCL/IPC need it)
    out.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if env_file and os.path.isfile(env_file):
        with open(env_file) as f:
            for raw in f:
                line = raw.strip()
                if line and not line.startswith("#") and "=" in line:
                    k, v = line.split("=", 1)
                    out[k.strip()] = v.strip()
    return out


def child_env(base: dict[str, str], info: RankInfo, world: int, local_world: int, master_addr: str,
              master_port: int) -> dict[str, str]:
    env = dict(base)
    env.update({"RANK": str(info.rank), "LOCAL_RANK": str(info.local_rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(local_world), "NODE_RANK": str(info.node_rank),
                "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port),
                "DTD_DEVICE": str(info.device)})
    return env


def child_cmd(cmd: list[str], info: RankInfo, append_local_rank: bool, module: bool = False) -> list[str]:
    exe = [sys.executable, "-u"] + (["-m"] if module else []) + list(cmd)
    if append_local_rank:
        exe.append(f"--local_rank={info.local_rank}")
    return exe


class NodeAgent:
    """Starts and supervises this node's ranks.  ``run()`` returns the job's exit code."""

    def __init__(self, hosts: list[Host], node_rank: int, master_addr: str, master_port: int, cmd: list[str],
                 append_local_rank: bool = True, module: bool = False, env: dict[str, str] | None = None,
                 poll_s: float = 0.1):
        self.table = [r for r in rank_table(hosts) if r.node_rank == node_rank]
        self.world = sum(h.slots for h in hosts)
        self.local_world = hosts[node_rank].slots
        self.master_addr, self.master_port = master_addr, master_port
        self.cmd, self.append_local_rank, self.module = cmd, append_local_rank, module
        self.env = dict(os.environ if env is None else env)
        self.poll_s = poll_s
        self.procs: list[subprocess.Popen] = []

    def commands(self) -> list[tuple[list[str], dict[str, str]]]:
        return [(child_cmd(self.cmd, r, self.append_local_rank, self.module),
                 child_env(self.env, r, self.world, self.local_world, self.master_addr, self.master_port))
                for r in self.table]

    def _terminate(self, sig=signal.SIGTERM, grace_s: float = 10.0):
        for p in self.procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)        # the child's own process group (start_new_session)
                except ProcessLookupError:
                    pass
        deadline = time.time() + grace_s
        for p in self.procs:
            try:
                p.wait(timeout=max(0.0, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    def run(self) -> int:
        for cmd, env in self.commands():
            self.procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
        prev = {s: signal.getsignal(s) for s in (signal.SIGINT, signal.SIGTERM)}

        def _forward(signum, _frame):
            self._terminate(signum)
            raise SystemExit(128 + signum)
        for s in prev:
            signal.signal(s, _forward)
        try:
            while True:
                codes = [p.poll() for p in self.procs]
                failed = [c for c in codes if c not in (None, 0)]
                if failed:
                    self._terminate()
                    return failed[0] if failed[0] > 0 else 128 - failed[0]
                if all(c == 0 for c in codes):
                    return 0
                time.sleep(self.poll_s)
        finally:
            for s, h in prev.items():
                signal.signal(s, h)


def ssh_command(host: str, node_rank: int, hostfile_arg: str, master_addr: str, master_port: int, cmd: list[str],
                env: dict[str, str], workdir: str, extra: list[str], ssh_port: int | None = None) -> list[str]:
    """The ``ssh`` line that starts node ``node_rank``'s agent on ``host``."""
    exports = " ".join(f"export {k}={shlex.quote(v)};" for k, v in sorted(env.items()))
    agent = [sys.executable, "-u", "-m", "distributed_training_and_deepspeed_amd.launch.multinode",
             "--hostfile", hostfile_arg, "--node-rank", str(node_rank), "--master-addr", master_addr,
             "--master-port", str(master_port)] + extra + ["--"] + list(cmd)
    remote = f"cd {shlex.quote(workdir)}; {exports} " + " ".join(shlex.quote(a) for a in agent)
    base = ["ssh", "-o", "BatchMode=yes", "-o", "StrictHostKeyChecking=accept-new"]
    if ssh_port:
        base += ["-p", str(ssh_port)]
    return base + [host, remote]


def _parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Launch one process per MI355X across the nodes of a hostfile.")
    p.add_argument("--hostfile", default="", help="'host slots=N' lines; default: this host only")
    p.add_argument("--include", default="", help="host1:0,1@host2 -- restrict to these hosts/slots")
    p.add_argument("--exclude", default="", help="host1:3@host2 -- drop these hosts/slots")
    p.add_argument("--num-nodes", "--num_nodes", type=int, default=-1)
    p.add_argument("--num-gpus", "--num_gpus", "--nproc-per-node", type=int, default=-1)
    p.add_argument("--master-addr", "--master_addr", default="", help="default: first host in the hostfile")
    p.add_argument("--master-port", "--master_port", type=int, default=29500)
    p.add_argument("--node-rank", type=int, default=-1, help="(internal) run only this node's agent")
    p.add_argument("--ssh-port", type=int, default=None)
    p.add_argument("--no-local-rank", action="store_true", help="do not append --local_rank=i to the script")
    p.add_argument("--module", "-m", action="store_true", help="the target is a python module")
    p.add_argument("--dry-run", action="store_true", help="print the per-node commands and exit")
    p.add_argument("cmd", nargs=argparse.REMAINDER, help="script.py [script args]")
    return p


def _local_hosts(num_gpus: int) -> list[Host]:
    n = num_gpus
    if n <= 0:
        try:
            import torch
            n = max(1, torch.cuda.device_count())
        except Exception:  # noqa: BLE001
            n = 1
    return [Host("localhost", n)]


def main(argv: list[str] | None = None) -> int:
    a = _parser().parse_args(argv)
    cmd = a.cmd[1:] if a.cmd[:1] == ["--"] else a.cmd
    if not cmd:
        raise SystemExit("no script given")
    if a.hostfile:
        with open(a.hostfile) as f:
            hosts = parse_hostfile(f.read())
    else:
        hosts = _local_hosts(a.num_gpus)
    hosts = select_hosts(hosts, a.include, a.exclude, a.num_nodes, a.num_gpus)
    master = a.master_addr or ("127.0.0.1" if is_local(hosts[0].name) else hosts[0].name)
    append = not a.no_local_rank
    if a.node_rank >= 0:                          # agent mode (started by ssh, or local single node)
        return NodeAgent(hosts, a.node_rank, master, a.master_port, cmd, append, a.module).run()
    if len(hosts) == 1 and is_local(hosts[0].name):
        agent = NodeAgent(hosts, 0, master, a.master_port, cmd, append, a.module)
        if a.dry_run:
            for c, e in agent.commands():
                print(" ".join(f"{k}={e[k]}" for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                        "MASTER_PORT")), " ".join(c))
            return 0
        return agent.run()
    env = forwarded_env()
    extra = [f"--num-gpus={a.num_gpus}"] if a.num_gpus > 0 else []
    if a.include:
        extra.append(f"--include={a.include}")
    if a.exclude:
        extra.append(f"--exclude={a.exclude}")
    if a.num_nodes > 0:
        extra.append(f"--num-nodes={a.num_nodes}")
    if a.no_local_rank:
        extra.append("--no-local-rank")
    if a.module:
        extra.append("--module")
    hostfile_arg = os.path.abspath(a.hostfile)
    lines = [ssh_command(h.name, n, hostfile_arg, master, a.master_port, cmd, env, os.getcwd(), extra, a.ssh_port)
             for n, h in enumerate(hosts)]
    if a.dry_run:
        for ln in lines:
            print(" ".join(shlex.quote(x) for x in ln))
        return 0
    procs = [subprocess.Popen(ln, start_new_session=True) for ln in lines]
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0] if bad[0] > 0 else 1
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.2)
    finally:
        for p in procs:                            # tear down the remaining ssh sessions (and their agents)
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
    return rc


if __name__ == "__main__":
    sys.exit(main())
