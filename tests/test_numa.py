"""NUMA-aware rank placement (runtime/numa.py) against a fake sysfs tree, and
the deferred, consumer-initialised request rings (Job.init_req_ring)."""
import os

import pytest

from ray_dynamic_batching_amd.runtime import numa


def _fake_sysfs(tmp_path, gpus):
    """gpus: [(bdf, node, cpulist or None)]; two NUMA nodes of 8 CPUs."""
    root = tmp_path / "sys"
    for n, cl in ((0, "0-7"), (1, "8-15")):
        d = root / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cl + "\n")
    kfd = root / "class" / "kfd" / "kfd" / "topology" / "nodes"
    (kfd / "0").mkdir(parents=True)
    (kfd / "0" / "properties").write_text("cpu_cores_count 16\nsimd_count 0\nlocation_id 0\n")
    for i, (bdf, node, cl) in enumerate(gpus):
        d = root / "bus" / "pci" / "devices" / bdf
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{node}\n")
        if cl is not None:
            (d / "local_cpulist").write_text(cl + "\n")
        dom, bus, rest = bdf.split(":")
        dev, fn = rest.split(".")
        loc = (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn)
        k = kfd / str(i + 1)
        k.mkdir()
        (k / "properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {loc}\ndomain {int(dom, 16)}\n")
    return str(root)


GPUS8 = [(f"0000:{b:02x}:00.0", 0 if i < 4 else 1, None if i % 2 else ("0-7" if i < 4 else "8-15"))
         for i, b in enumerate([0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xe5, 0xf5])]


def test_cpulist_roundtrip():
    assert numa.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert numa.format_cpulist([11, 10, 0, 1, 2, 3, 8]) == "0-3,8,10-11"
    assert numa.parse_cpulist("") == []


def test_kfd_order_and_pci_locality(tmp_path, monkeypatch):
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    sysfs = _fake_sysfs(tmp_path, GPUS8)
    pci = numa.kfd_gpu_pci_addresses(sysfs)
    assert pci == [g[0] for g in GPUS8]
    assert numa.pci_locality(pci[0], sysfs) == (0, list(range(8)))
    assert numa.pci_locality(pci[1], sysfs) == (0, list(range(8)))       # no local_cpulist: node's cpulist
    assert numa.pci_locality(pci[7], sysfs) == (1, list(range(8, 16)))
    assert numa.pci_locality("0000:ff:00.0", sysfs) == (-1, [])          # absent: no pinning
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "6,1")
    assert numa.kfd_gpu_pci_addresses(sysfs) == [GPUS8[6][0], GPUS8[1][0]]


def test_eight_ranks_get_distinct_socket_local_cpu_sets(tmp_path, monkeypatch):
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    sysfs = _fake_sysfs(tmp_path, GPUS8)
    loc = numa.gpu_locality_map(sysfs, numa.kfd_gpu_pci_addresses(sysfs))
    sets = numa.plan_cpu_sets(list(range(8)), loc)
    assert sets == [[0, 1], [2, 3], [4, 5], [6, 7], [8, 9], [10, 11], [12, 13], [14, 15]]
    flat = [c for s in sets for c in s]
    assert len(flat) == len(set(flat)) == 16
    # the cgroup's allowed CPUs are respected
    sets = numa.plan_cpu_sets(list(range(8)), loc, allowed=range(0, 16, 2))
    assert sets[:4] == [[0], [2], [4], [6]] and sets[4:] == [[8], [10], [12], [14]]
    # 8 ranks rehearsed on ONE GPU split that GPU's node
    sets = numa.plan_cpu_sets([0] * 8, loc)
    assert sets == [[c] for c in range(8)]
    # unknown locality: no pinning
    assert numa.plan_cpu_sets([0, 1], {}) == [[], []]


def test_place_rank_pins_this_process(tmp_path, monkeypatch):
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    have = sorted(os.sched_getaffinity(0))
    if len(have) < 2:
        pytest.skip("needs >= 2 CPUs")
    sysfs = _fake_sysfs(tmp_path, [("0000:05:00.0", 0, numa.format_cpulist(have)),
                                   ("0000:15:00.0", 0, numa.format_cpulist(have))])
    try:
        out = numa.place_rank(1, [0, 1], sysfs=sysfs)
        assert out["pinned"] and out["numa_node"] == 0
        mine = numa.parse_cpulist(out["cpus"])
        assert set(os.sched_getaffinity(0)) == set(mine)
        assert mine == have[len(have) - len(mine):]                        # rank 1: the second half
    finally:
        os.sched_setaffinity(0, set(have))
    monkeypatch.setenv("RDB_NUMA_PIN", "0")
    assert numa.place_rank(0, [0], sysfs=sysfs)["pinned"] is False


def test_deferred_request_rings_are_initialised_by_their_consumer():
    from ray_dynamic_batching_amd.runtime import job as rjob

    name = rjob.unique_job_name("numa")
    j = rjob.Job(name, create=True, n_replicas=2, n_queues=2, n_clients=2, req_capacity=64, defer_req_rings=True)
    j.unlink_on_close(True)
    assert j.init_req_ring(0, 0) in (0, -1, -22, -38)         # mbind may be refused in a container
    assert j.init_req_ring(1, -1) == 0
    j.configure_queue(0, 0, 0, 16)
    j.configure_queue(1, 1, 0, 16)
    cli = rjob.Client(j)
    cons = rjob.Consumer(j, [0, 1])
    for q in (0, 1):
        for i in range(70):                                   # wraps the 64-slot ring
            assert cli.submit(q, b"p%d" % i) >= 0
            got = cons.pop(4, 0)
            assert [g[6] for g in got] == [b"p%d" % i]
    j.close()
