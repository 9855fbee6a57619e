"""Cluster description -> hostfile, ssh config and RCCL environment for multi-node MI355X jobs.

The reference provisions its clusters with AWS CDK (aws/training_stack.py:9-29 one g4dn.12xlarge;
aws/multi_node_training_stack.py:9-50 three g4dn.xlarge in one security group with all intra-group
traffic allowed for NCCL sockets) and its outputs are (a) the hostfile text
``"<dns> slots=1"`` (multi_node_training_stack.py:40-41) and (b) an ssh-config block ``worker-1..3``
(:44-49) that scripts/generate-keys.sh (R15) installs on every worker.

MI355X nodes are not provisioned through a cloud SDK in this image (no aws-cdk, no network), so the
equivalent here starts from an *inventory* (YAML/JSON: node names, addresses, GPUs per node, NIC
settings) and renders the same artefacts, sized for 8x MI355X per node:

* ``hostfile()``        -- ``worker-1 slots=8`` lines for ``launch/multinode.py``;
* ``ssh_config()``      -- ``Host worker-i / HostName / User / IdentityFile`` blocks;
* ``rccl_env()``        -- the ``.dtd_env`` lines the launcher forwards: dmabuf IPC
  (``HSA_ENABLE_IPC_MODE_LEGACY=0``), the inter-node NIC (``NCCL_SOCKET_IFNAME`` / ``NCCL_IB_HCA``),
  and enough RCCL channels that intra-node rings spread over all 7 xGMI links per GPU;
* ``firewall_note()``   -- the port ranges that must be open between nodes (the SG rule of the
  reference's stack: TCPStore master port + RCCL's bootstrap/socket ports).

``python -m distributed_training_and_deepspeed_amd.launch.cluster inventory.yaml --out-dir cluster/``
writes ``hostfile``, ``ssh_config`` and ``.dtd_env``.
"""
from __future__ import annotations

import argparse
import json
import os
from dataclasses import dataclass, field

import yaml


@dataclass
class Node:
    name: str
    address: str
    gpus: int = 8


@dataclass
class Cluster:
    name: str
    nodes: list[Node]
    user: str = "root"
    ssh_key: str = "~/.ssh/dtd_cluster"
    master_port: int = 29500
    socket_ifname: str = ""        # e.g. "ens" / "bond0": inter-node bootstrap + socket transport
    ib_hca: str = ""               # RoCE/IB HCA list for RCCL's IB transport, e.g. "mlx5_0,mlx5_1"
    min_channels: int = 32         # >= 4 rings per xGMI link pair; RCCL's default can leave links idle
    extra_env: dict[str, str] = field(default_factory=dict)

    @classmethod
    def from_dict(cls, d: dict) -> "Cluster":
        gpus = int(d.get("gpus_per_node", 8))
        nodes = []
        for i, n in enumerate(d.get("nodes", []), 1):
            if isinstance(n, str):
                n = {"address": n}
            nodes.append(Node(n.get("name", f"worker-{i}"), n["address"], int(n.get("gpus", gpus))))
        if not nodes:
            raise ValueError("inventory has no nodes")
        names = [n.name for n in nodes]
        if len(set(names)) != len(names):
            raise ValueError(f"duplicate node names in inventory: {names}")
        net = d.get("network", {}) or {}
        return cls(name=d.get("cluster", "mi355x"), nodes=nodes, user=d.get("user", "root"),
                   ssh_key=d.get("ssh_key", "~/.ssh/dtd_cluster"), master_port=int(d.get("master_port", 29500)),
                   socket_ifname=net.get("socket_ifname", ""), ib_hca=net.get("ib_hca", ""),
                   min_channels=int(net.get("min_channels", 32)), extra_env=dict(d.get("env", {}) or {}))

    @classmethod
    def load(cls, path: str) -> "Cluster":
        with open(path) as f:
            text = f.read()
        d = json.loads(text) if path.endswith(".json") else yaml.safe_load(text)
        return cls.from_dict(d)

    @property
    def world_size(self) -> int:
        return sum(n.gpus for n in self.nodes)

    def hostfile(self) -> str:
        return "".join(f"{n.name} slots={n.gpus}\n" for n in self.nodes)

    def ssh_config(self) -> str:
        blocks = []
        for n in self.nodes:
            blocks.append(f"Host {n.name}\n    HostName {n.address}\n    User {self.user}\n"
                          f"    IdentityFile {self.ssh_key}\n    StrictHostKeyChecking accept-new\n")
        return "\n".join(blocks)

    def rccl_env(self) -> dict[str, str]:
        env = {"HSA_ENABLE_IPC_MODE_LEGACY": "0", "NCCL_MIN_NCHANNELS": str(self.min_channels),
               "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1"}
        if self.socket_ifname:
            env["NCCL_SOCKET_IFNAME"] = self.socket_ifname
            env["GLOO_SOCKET_IFNAME"] = self.socket_ifname
        if self.ib_hca:
            env["NCCL_IB_HCA"] = self.ib_hca
        env.update(self.extra_env)
        return env

    def firewall_note(self) -> str:
        return (f"allow all TCP between cluster nodes (TCPStore on {self.nodes[0].name}:{self.master_port}, "
                "RCCL bootstrap and socket transport use ephemeral ports), plus ssh (22) from the launch host")

    def write(self, out_dir: str) -> list[str]:
        os.makedirs(out_dir, exist_ok=True)
        files = {"hostfile": self.hostfile(), "ssh_config": self.ssh_config(),
                 ".dtd_env": "".join(f"{k}={v}\n" for k, v in self.rccl_env().items())}
        paths = []
        for name, text in files.items():
            p = os.path.join(out_dir, name)
            with open(p, "w") as f:
                f.write(text)
            paths.append(p)
        return paths


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="Render hostfile / ssh config / RCCL env from a cluster inventory.")
    p.add_argument("inventory")
    p.add_argument("--out-dir", default="cluster")
    a = p.parse_args(argv)
    c = Cluster.load(a.inventory)
    for path in c.write(a.out_dir):
        print("wrote", path)
    print(f"{c.name}: {len(c.nodes)} nodes, world size {c.world_size}; {c.firewall_note()}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
