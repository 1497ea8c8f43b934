"""NUMA placement of the library's threads (numa.c): the CPUs chosen for a GPU from a fake
sysfs tree — the node from /sys/bus/pci/devices/<bus id>/numa_node, its CPUs from
/sys/devices/system/node/node<n>/cpulist, intersected with the process's affinity."""
import ctypes
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUS = "0000:05:00.0"


def _lib():
    L = ctypes.CDLL(os.path.join(ROOT, "m2dec_amd", "lib", "libm2dec_amd.so"))
    L.m2dec_amd_numa_cpus.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_int)]
    return L


def _sysfs(tmp_path, node, cpulists, bus=BUS):
    d = tmp_path / "sys" / "bus" / "pci" / "devices" / bus
    d.mkdir(parents=True)
    (d / "numa_node").write_text(f"{node}\n")
    for n, cl in cpulists.items():
        nd = tmp_path / "sys" / "devices" / "system" / "node" / f"node{n}"
        nd.mkdir(parents=True)
        (nd / "cpulist").write_text(cl + "\n")
    return str(tmp_path)


def _cpus(L, root, bus):
    buf = (ctypes.c_int * 1024)()
    node = ctypes.c_int()
    k = L.m2dec_amd_numa_cpus(root.encode(), bus.encode(), buf, 1024, ctypes.byref(node))
    return node.value, set(buf[:k])


def test_node_cpus_intersected_with_affinity(built, tmp_path):
    allowed = os.sched_getaffinity(0)
    some = sorted(allowed)[: max(1, len(allowed) // 2)]
    # node 1 holds half of this process's CPUs and CPUs it may not use
    cl = ",".join(str(c) for c in some) + ",1020-1023"
    root = _sysfs(tmp_path, 1, {0: "0-1", 1: cl})
    node, got = _cpus(_lib(), root, BUS.upper())  # (hipDeviceGetPCIBusId may give upper case)
    assert node == 1
    assert got == set(some)


def test_unknown_node_keeps_the_affinity(built, tmp_path):
    root = _sysfs(tmp_path, -1, {0: "0-3"})
    node, got = _cpus(_lib(), root, BUS)
    assert node == -1
    assert got == os.sched_getaffinity(0)
    node, got = _cpus(_lib(), str(tmp_path / "nowhere"), BUS)
    assert node == -1 and got == os.sched_getaffinity(0)


def test_node_outside_the_affinity_keeps_it(built, tmp_path):
    root = _sysfs(tmp_path, 3, {3: "1000-1010"})
    node, got = _cpus(_lib(), root, BUS)
    assert node == 3
    assert got == os.sched_getaffinity(0)


@pytest.mark.parametrize("cl, want", [("0-3,8,10-11", {0, 1, 2, 3, 8, 10, 11}), ("5", {5})])
def test_cpulist_parsing(built, tmp_path, cl, want):
    root = _sysfs(tmp_path, 0, {0: cl})
    node, got = _cpus(_lib(), root, BUS)
    assert node == 0
    assert got == want & os.sched_getaffinity(0) or got == os.sched_getaffinity(0)


def test_one_thread_per_core(built, tmp_path, monkeypatch):
    """M2DEC_AMD_NUMA_SMT=1: of each core's sibling hardware threads only the lowest is kept."""
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 4:
        pytest.skip("needs 4 CPUs")
    a, b, c, d = allowed[:4]
    root = _sysfs(tmp_path, 0, {0: f"{a},{b},{c},{d}"})
    for cpu, sib in ((a, f"{a},{c}"), (c, f"{a},{c}"), (b, f"{b},{d}"), (d, f"{b},{d}")):
        t = tmp_path / "sys" / "devices" / "system" / "cpu" / f"cpu{cpu}" / "topology"
        t.mkdir(parents=True)
        (t / "thread_siblings_list").write_text(sib + "\n")
    monkeypatch.setenv("M2DEC_AMD_NUMA_SMT", "1")
    node, got = _cpus(_lib(), root, BUS)
    assert node == 0 and got == {a, b}
    monkeypatch.setenv("M2DEC_AMD_NUMA_SMT", "0")
    node, got = _cpus(_lib(), root, BUS)
    assert got == {a, b, c, d}
