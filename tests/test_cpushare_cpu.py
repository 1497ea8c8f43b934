"""The host CPU share (cpushare.c): affinity ∩ the cgroup quota ÷ the node's GPU ranks, from
fake /proc + cgroup trees; the library's parse pool, MD5 threads and H.265 workers sized by it; the per-rank CPU
plan of m2dec_amd.dist for 8 ranks on a fake 2-node machine (disjoint CPU sets, shares within the quota)."""
import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib():
    L = ctypes.CDLL(os.path.join(ROOT, "m2dec_amd", "lib", "libm2dec_amd.so"))
    L.m2dec_amd_cpu_share.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_long),
                                      ctypes.POINTER(ctypes.c_int)]
    return L


def _share(root, ranks, aff):
    q, a = ctypes.c_long(), ctypes.c_int()
    s = _lib().m2dec_amd_cpu_share(str(root).encode(), ranks, aff, ctypes.byref(q), ctypes.byref(a))
    return s, q.value


def _v2(tmp_path, cg, levels):
    """cgroup v2: /proc/self/cgroup = 0::cg, cpu.max per directory (levels: {relative dir: text})."""
    (tmp_path / "proc" / "self").mkdir(parents=True)
    (tmp_path / "proc" / "self" / "cgroup").write_text(f"0::{cg}\n")
    for d, txt in levels.items():
        p = tmp_path / "sys" / "fs" / "cgroup" / d
        p.mkdir(parents=True, exist_ok=True)
        (p / "cpu.max").write_text(txt + "\n")
    return tmp_path


def test_v2_quota_of_the_job(built, tmp_path):
    root = _v2(tmp_path, "/jobs/j1", {"": "max 100000", "jobs": "max 100000", "jobs/j1": "1600000 100000"})
    assert _share(root, 1, 256) == (16, 16000)      # the GPU box: 16 CPUs of quota over a 256-CPU mask
    assert _share(root, 1, 8) == (8, 16000)         # a narrower affinity wins
    assert _share(root, 8, 256) == (2, 16000)       # one job's quota over 8 GPU ranks
    assert _share(root, 8, 24) == (2, 16000)


def test_v2_tighter_ancestor(built, tmp_path):
    root = _v2(tmp_path, "/a/b", {"": "max 100000", "a": "400000 100000", "a/b": "max 100000"})
    assert _share(root, 1, 64) == (4, 4000)


def test_v2_fractional_and_container_root(built, tmp_path):
    root = _v2(tmp_path, "/", {"": "250000 100000"})  # a container sees its cgroup as the mount's root
    assert _share(root, 1, 64) == (2, 2500)


def test_v1_cfs_quota(built, tmp_path):
    (tmp_path / "proc" / "self").mkdir(parents=True)
    (tmp_path / "proc" / "self" / "cgroup").write_text("3:cpuset:/jobs\n2:cpu,cpuacct:/x\n0::/\n")
    d = tmp_path / "sys" / "fs" / "cgroup" / "cpu,cpuacct" / "x"
    d.mkdir(parents=True)
    (d / "cpu.cfs_quota_us").write_text("800000\n")
    (d / "cpu.cfs_period_us").write_text("100000\n")
    assert _share(tmp_path, 1, 32) == (8, 8000)


def test_no_quota(built, tmp_path):
    root = _v2(tmp_path, "/", {"": "max 100000"})
    assert _share(root, 1, 12) == (12, -1)
    c = tmp_path / "sys" / "devices" / "system" / "cpu"
    c.mkdir(parents=True)
    (c / "online").write_text("0-63,64-127\n")
    assert _share(root, 4, 128) == (32, -1)  # the whole machine, unpinned: split among the ranks
    assert _share(root, 4, 24) == (24, -1)   # a pinned rank keeps its own mask
    assert _share(tmp_path / "nowhere", 1, 6) == (6, -1)


def _threads_of(env_extra, code):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip().splitlines()[-1]


_COUNT = r"""
import ctypes, os, sys
sys.path.insert(0, '.')
import m2dec_amd
from tests._oracle import OracleBackend
from tests._streams import stream
data = stream('cov_cabac_s1')
with OracleBackend() as ob:
    m2dec_amd.decode_stream_md5_backend(data, ob.be, parse_threads=2, md5_threads=2)
names = [open(f'/proc/self/task/{t}/comm').read().strip() for t in os.listdir('/proc/self/task')]
L = m2dec_amd.lib()
sl = ctypes.c_int()
share = L.m2dec_amd_cpu_gate(ctypes.byref(sl), None, None, None)
print(share, sl.value, sum(n == 'm2d-parse' for n in names), sum(n == 'm2d-copy' for n in names))
"""


@pytest.mark.parametrize("share, slots, crew", [(4, 4, 1), (12, 11, 3), (16, 15, 3)])
def test_pool_sized_by_the_share(built, share, slots, crew):
    out = _threads_of({"M2DEC_AMD_CPU_SHARE": str(share)}, _COUNT).split()
    s, sl, parse, copy = map(int, out)
    assert (s, sl) == (share, slots)
    assert parse == slots  # the parse pool: one worker per busy-thread slot
    assert copy <= 2 * crew  # two crews (submission, sync), each at most `crew` helpers


def test_affinity_sets_the_share(built):
    cpus = sorted(os.sched_getaffinity(0))[:3]
    code = f"import os; os.sched_setaffinity(0, {cpus!r}); exec(open('/dev/stdin').read())"
    env = dict(os.environ)
    env.pop("M2DEC_AMD_CPU_SHARE", None)
    r = subprocess.run([sys.executable, "-c", code], input=_COUNT, cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    s, sl, parse, _ = map(int, r.stdout.strip().splitlines()[-1].split())
    assert s == len(cpus) and sl == len(cpus) and parse == len(cpus)


def _two_nodes(tmp_path, gpus_per_node=4, cpus_per_node=64, quota=None):
    """A fake 2-socket, 8-GPU node: GPUs 0000:0<g>:00.0, the first four on node 0, CPUs 0-63 / 64-127."""
    c = tmp_path / "sys" / "devices" / "system" / "cpu"
    c.mkdir(parents=True)
    (c / "online").write_text(f"0-{2 * cpus_per_node - 1}\n")
    for n in range(2):
        d = tmp_path / "sys" / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(f"{n * cpus_per_node}-{(n + 1) * cpus_per_node - 1}\n")
    buses = []
    for g in range(2 * gpus_per_node):
        b = f"0000:{0x10 + g:02x}:00.0"
        d = tmp_path / "sys" / "bus" / "pci" / "devices" / b
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{g // gpus_per_node}\n")
        buses.append(b)
    if quota:
        _v2(tmp_path, "/", {"": f"{quota * 100000} 100000"})
    return str(tmp_path), buses


def test_eight_ranks_get_disjoint_cpus_and_shares_within_the_quota(built, tmp_path):
    """8 simulated ranks on a fake 2-node machine (m2dec_amd.dist.cpu_plan, what place_rank
    applies under torchrun): disjoint CPU sets on their GPU's node, equal per node; each rank's library share
    (cpushare.c) within the job's quota ÷ 8.  Unmeasured on an 8-GPU node."""
    import m2dec_amd.dist as md
    for quota, want_share in ((None, 16), (64, 8), (128, 16), (16, 2)):
        sub = tmp_path / f"q{quota}"
        sub.mkdir()
        root, buses = _two_nodes(sub, quota=quota)
        nodes = [md.gpu_numa_node(b.upper(), root) for b in buses]
        assert nodes == [0, 0, 0, 0, 1, 1, 1, 1]
        plan = md.cpu_plan(nodes, md.node_cpus(root), range(128))
        seen = set()
        for r, cpus in enumerate(plan):
            assert len(cpus) == 16 and not (seen & set(cpus))
            seen |= set(cpus)
            node_range = range(64 * nodes[r], 64 * nodes[r] + 64)
            assert all(c in node_range for c in cpus)
            share, q = _share(root, 8, len(cpus))
            assert share == want_share and (q == -1 if quota is None else q == quota * 1000)
            assert share * 8 <= (quota or 128)


def test_cpu_plan_fallbacks():
    import m2dec_amd.dist as md
    # a node outside the job's affinity: split everything allowed among all ranks
    p = md.cpu_plan([0, 1], {0: list(range(8)), 1: list(range(8, 16))}, range(8))
    assert p == [[0, 1, 2, 3], [4, 5, 6, 7]]
    # unknown node
    assert md.cpu_plan([-1, -1, -1], {}, [3, 4, 5, 6, 7, 8]) == [[3, 4], [5, 6], [7, 8]]
    # fewer CPUs than ranks: one each, round robin
    assert md.cpu_plan([0, 0, 0], {0: [0, 1]}, range(2)) == [[0], [1], [0]]
    assert md.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
