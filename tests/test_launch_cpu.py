"""Multi-node launcher (DeepSpeed-runner parity): hostfile law, filters, rank
table, ssh fan-out line, local agent with fail-fast."""
import json
import os
import time

import pytest

from distributed_training_and_deepspeed_amd.launch import multinode as M

HOSTFILE = """
# three MI355X nodes
node-a slots=8
node-b slots=8   # trailing comment
node-c slots=4
"""
TARGET = os.path.join(os.path.dirname(__file__), "helpers", "launch_target.py")


def test_parse_hostfile():
    hosts = M.parse_hostfile(HOSTFILE)
    assert [(h.name, h.slots) for h in hosts] == [("node-a", 8), ("node-b", 8), ("node-c", 4)]
    with pytest.raises(ValueError):
        M.parse_hostfile("a slots=2\na slots=2")
    with pytest.raises(ValueError):
        M.parse_hostfile("a")
    with pytest.raises(ValueError):
        M.parse_hostfile("# nothing\n")


def test_filters_and_rank_table():
    hosts = M.parse_hostfile(HOSTFILE)
    sel = M.select_hosts(hosts, include="node-a:0,1@node-c")
    assert [(h.name, h.devices) for h in sel] == [("node-a", [0, 1]), ("node-c", [0, 1, 2, 3])]
    sel = M.select_hosts(hosts, exclude="node-b@node-c:3")
    assert [(h.name, h.slots) for h in sel] == [("node-a", 8), ("node-c", 3)]
    sel = M.select_hosts(hosts, num_nodes=2, num_gpus=2)
    t = M.rank_table(sel)
    assert [(r.host, r.node_rank, r.local_rank, r.rank) for r in t] == [
        ("node-a", 0, 0, 0), ("node-a", 0, 1, 1), ("node-b", 1, 0, 2), ("node-b", 1, 1, 3)]
    with pytest.raises(ValueError):
        M.select_hosts(hosts, include="node-z")
    with pytest.raises(ValueError):
        M.select_hosts(hosts, include="node-a", exclude="node-b")


def test_ssh_line_resolves_master_locally(tmp_path):
    hf = tmp_path / "hostfile"
    hf.write_text(HOSTFILE)
    env = {"NCCL_DEBUG": "WARN", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    line = M.ssh_command("node-b", 1, str(hf), "node-a", 29500, ["zero_dp_training.py", "--stage=2"], env,
                         "/work", ["--num-gpus=8"])
    assert line[:1] == ["ssh"] and "node-b" in line
    remote = line[-1]
    assert "export NCCL_DEBUG=WARN;" in remote and "--master-addr node-a" in remote
    assert "--node-rank 1" in remote and remote.rstrip().endswith("zero_dp_training.py --stage=2")


def test_forwarded_env_keeps_dmabuf_ipc(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    (tmp_path / M.ENV_FILE).write_text("NCCL_MIN_NCHANNELS=32\n# c\nFOO=bar\n")
    env = M.forwarded_env({"NCCL_ALGO": "Ring", "HOME": "/root"})
    assert env["NCCL_ALGO"] == "Ring" and "HOME" not in env
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["NCCL_MIN_NCHANNELS"] == "32" and env["FOO"] == "bar"


def test_local_agent_runs_two_ranks(tmp_path):
    port = M.socket.socket()
    port.bind(("127.0.0.1", 0))
    p = port.getsockname()[1]
    port.close()
    rc = M.main(["--num-gpus", "2", "--master-port", str(p), TARGET, "--out", str(tmp_path)])
    assert rc == 0
    res = [json.loads((tmp_path / f"r{r}.json").read_text()) for r in range(2)]
    assert all(r["sum"] == 3.0 for r in res)
    assert [r["local_rank"] for r in res] == [0, 1]
    assert all(r["unknown"] == [f"--local_rank={i}"] for i, r in enumerate(res))   # DeepSpeed convention
    assert all(r["local_world"] == 2 and r["node_rank"] == 0 for r in res)


def test_fail_fast_terminates_siblings(tmp_path):
    t0 = time.time()
    rc = M.main(["--num-gpus", "3", "--master-port", "29999", TARGET, "--out", str(tmp_path), "--fail-rank", "1"])
    assert rc == 3
    assert time.time() - t0 < 60   # siblings (sleeping 120 s) were killed


def test_cluster_inventory_renders_launcher_files(tmp_path):
    from distributed_training_and_deepspeed_amd.launch.cluster import Cluster
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    c = Cluster.load(os.path.join(root, "infra", "mi355x_cluster.example.yaml"))
    assert c.world_size == 16
    c.write(str(tmp_path))
    hosts = M.parse_hostfile((tmp_path / "hostfile").read_text())
    assert [(h.name, h.slots) for h in hosts] == [("worker-1", 8), ("worker-2", 8)]
    assert "HostName 10.0.0.12" in (tmp_path / "ssh_config").read_text()
    env = (tmp_path / ".dtd_env").read_text()
    assert "HSA_ENABLE_IPC_MODE_LEGACY=0" in env and "NCCL_SOCKET_IFNAME=bond0" in env
