"""Host placement of one-process-per-GPU ranks (triton_client_amd/parallel/placement.py)
on a fake two-socket sysfs tree: 8 GPUs, four on each NUMA node."""

import os

import pytest

from triton_client_amd.parallel import placement


def _fake_host(root, gpu_nodes, node_cpus):
    """KFD topology (CPU nodes first, then one node per GPU), PCI numa_node
    files and the NUMA nodes' cpulists."""
    kfd = root / "sys/class/kfd/kfd/topology/nodes"
    n = 0
    for _ in node_cpus:  # CPU agents: simd_count 0
        (kfd / str(n)).mkdir(parents=True)
        (kfd / str(n) / "properties").write_text("cpu_cores_count 64\nsimd_count 0\nlocation_id 0\ndomain 0\n")
        n += 1
    for i, numa in enumerate(gpu_nodes):
        bus = 0x10 + 0x10 * i
        (kfd / str(n)).mkdir(parents=True)
        (kfd / str(n) / "properties").write_text(
            "cpu_cores_count 0\nsimd_count 1024\nlocation_id %d\ndomain 0\n" % (bus << 8))
        dev = root / "sys/bus/pci/devices" / ("0000:%02x:00.0" % bus)
        dev.mkdir(parents=True)
        (dev / "numa_node").write_text("%d\n" % numa)
        n += 1
    for k, cpus in enumerate(node_cpus):
        d = root / ("sys/devices/system/node/node%d" % k)
        d.mkdir(parents=True)
        d.joinpath("cpulist").write_text(cpus + "\n")
    return str(root)


def test_cpulist_round_trip():
    assert placement.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert placement.format_cpulist([11, 10, 8, 3, 2, 1, 0]) == "0-3,8,10-11"
    assert placement.parse_cpulist("") == []


def test_gpu_order_and_pci_addresses(tmp_path, monkeypatch):
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    root = _fake_host(tmp_path, [0, 0, 1, 1], ["0-7", "8-15"])
    assert placement.gpu_bdfs(root) == ["0000:10:00.0", "0000:20:00.0", "0000:30:00.0", "0000:40:00.0"]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,0")
    assert placement.gpu_bdfs(root) == ["0000:30:00.0", "0000:10:00.0"]
    # CUDA_VISIBLE_DEVICES is HIP's alias, used only when HIP_VISIBLE_DEVICES
    # is unset: with both set it must not filter a second time
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "1")
    assert placement.gpu_bdfs(root) == ["0000:30:00.0", "0000:10:00.0"]
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    assert placement.gpu_bdfs(root) == ["0000:20:00.0"]
    # ROCR filters first, HIP indexes what is left
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "3,1,2")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,0")
    assert placement.gpu_bdfs(root) == ["0000:30:00.0", "0000:40:00.0"]


def test_two_socket_eight_gpus(tmp_path, monkeypatch):
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    # GPUs 0-3 on socket 0 (CPUs 0-63), GPUs 4-7 on socket 1 (CPUs 64-127)
    root = _fake_host(tmp_path, [0, 0, 0, 0, 1, 1, 1, 1], ["0-63", "64-127"])
    allowed = set(range(128))
    plans = [placement.plan(r, 8, root=root, allowed=allowed) for r in range(8)]
    for r, p in enumerate(plans):
        assert p["source"] == "numa" and p["numa_node"] == (0 if r < 4 else 1)
        assert p["ranks_on_node"] == 4 and len(p["cpus"]) == 16
        assert all((c < 64) == (r < 4) for c in p["cpus"])  # never the other socket
    assert plans[0]["cpulist"] == "0-15" and plans[5]["cpulist"] == "80-95"
    sets = [set(p["cpus"]) for p in plans]
    assert all(not (a & b) for i, a in enumerate(sets) for b in sets[i + 1:])
    assert set().union(*sets) == allowed


def test_cgroup_limits_and_fallbacks(tmp_path, monkeypatch):
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    root = _fake_host(tmp_path, [0, 0, 1, 1], ["0-63", "64-127"])
    # a cpuset of 16 CPUs, 8 per socket: each node's two ranks split its 8
    allowed = set(range(56, 72))
    p = [placement.plan(r, 4, root=root, allowed=allowed) for r in range(4)]
    assert [x["cpulist"] for x in p] == ["56-59", "60-63", "64-67", "68-71"]
    # a node with none of the allowed CPUs: the even split of the allowed set
    q = placement.plan(0, 4, root=root, allowed=set(range(100, 108)))
    assert q["source"] == "even-split" and q["cpulist"] == "100-101"
    # no KFD topology at all (a container): even split, node -1
    e = placement.plan(3, 4, root=str(tmp_path / "nothing"), allowed=set(range(8)))
    assert e == {"cpus": [6, 7], "cpulist": "6-7", "numa_node": -1, "bdf": None, "ranks_on_node": 4,
                 "source": "even-split"}
    # more ranks than CPUs: every rank still gets one
    assert [placement.plan(r, 4, root=str(tmp_path / "x"), allowed={3, 5})["cpus"] for r in range(4)] == \
        [[3], [5], [3], [5]]


@pytest.mark.skipif(not hasattr(os, "sched_setaffinity"), reason="no sched_setaffinity")
def test_apply_pins_this_process():
    before = os.sched_getaffinity(0)
    try:
        cpu = min(before)
        p = placement.apply({"cpus": [cpu], "cpulist": str(cpu)})
        assert p["applied"] and os.sched_getaffinity(0) == {cpu}
    finally:
        os.sched_setaffinity(0, before)
