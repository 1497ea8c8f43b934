"""GPU twin of tests/test_boundary_cpu.py: the same M2Decoder-shaped harness (delete[] of the context,
frames deleted and reallocated inside the header callback, no release call) over the built-in HIP
back end, checked against the CPU oracle and the reference-pinned F1 goldens."""
import os

import pytest

from tests._streams import GOLDEN, stream
from tests.test_boundary_cpu import F1, ROOT, check_concat, gen, harness, iters
from tests._oracle import golden_md5s

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["fit", "more", "resize"])
def test_gpu_stream_switch_like_m2decoder(built, tmp_path, name):
    s = gen(tmp_path, name)
    _, alone = harness([s])                 # oracle
    cat = str(tmp_path / "cat.264")
    with open(cat, "wb") as f:
        f.write(open(F1, "rb").read() + open(s, "rb").read())
    lines, _ = harness([cat], oracle=False)  # HIP
    f1 = golden_md5s(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"))
    check_concat(lines, f1, alone)


def test_gpu_dropped_contexts_are_reclaimed(built, tmp_path):
    """1080p decoders dropped mid-stream (GPU work and copies still in flight) and small ones run to
    the end, 20 in all, no release call: frames exact, threads constant, registry bounded."""
    c3 = str(tmp_path / "c3.264")
    open(c3, "wb").write(stream("c3_1080p_s1"))
    gold = GOLDEN["c3_1080p_s1"]["md5"]
    f1 = golden_md5s(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"))
    # (dropped mid-stream, a context is reclaimed when its address is reused or, over the cap, once
    # idle for M2DEC_AMD_IDLE_EVICT_S: 0 here)
    lines, md5 = harness(["-n", "10", "-m", "9", c3, F1], oracle=False,
                         env={"M2DEC_AMD_MAX_CONTEXTS": "2", "M2DEC_AMD_IDLE_EVICT_S": "0"})
    st = iters(lines)
    assert len(st) == 10
    assert len({x["threads"] for x in st}) == 1
    assert max(x["contexts"] for x in st) <= 2
    for i in range(10):
        assert md5[18 * i:18 * i + 9] == gold[:9]
        assert md5[18 * i + 9:18 * i + 18] == f1[:9]
    lines, md5 = harness(["-n", "3", "-k", F1, c3], oracle=False, env={"M2DEC_AMD_MAX_CONTEXTS": "3"})
    assert md5 == (f1 + gold) * 3
    assert max(x["contexts"] for x in iters(lines)) <= 3


def test_gpu_resize_while_other_streams_run(built, tmp_path):
    """One stream grows its geometry mid-stream (F1 then a 352x288 stream: the driver's header callback
    hands the old frame block back to the process-wide pool and takes a bigger one) while three 1080p
    streams decode concurrently in the same process (m2dec_amd_decode_streams_md5) and may take that
    block from the pool at once: every 1080p frame, F1's frames before the reallocation and the second
    stream's frames stay exact (frames still in the DPB at the reallocation are undefined, as in the
    reference: tests/test_boundary_cpu.py)."""
    import m2dec_amd
    s = gen(tmp_path, "resize")
    _, alone = harness([s])                                  # oracle
    cat = open(F1, "rb").read() + open(s, "rb").read()
    catp = str(tmp_path / "cat.264")
    open(catp, "wb").write(cat)
    lines, _ = harness([catp])                               # oracle: where the reallocation falls
    frames = [ln for ln in lines if not ln.startswith("#iter")]
    assert "#realloc" in frames
    k = frames.index("#realloc")
    f1 = golden_md5s(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"))
    names = [f"c4_1080p_s{i}" for i in (2, 3, 4)]
    for rep in range(2):
        got = m2dec_amd.decode_streams([cat] + [stream(n) for n in names])
        assert len(got[0]) == len(f1) + len(alone), rep
        assert got[0][:k] == f1[:k], rep
        assert got[0][-len(alone):] == alone, rep
        for n, g in zip(names, got[1:]):
            assert g == GOLDEN[n]["md5"], (rep, n)


@pytest.mark.gpu
def test_gpu_budget_per_context_after_4k(built):
    """a context's admission numbers depend on its own geometry only.  A 1080p context reads
    the same capacity / cost / pictures per launch before and after a 4K decode in the same process (round 4
    kept the smallest capacity any context had registered, for the life of the process)."""
    import m2dec_amd
    c3 = stream("c3_1080p_s1")
    with m2dec_amd.HipBackend(0) as hb:
        assert m2dec_amd.decode_stream(c3, backend=hb.be) == GOLDEN["c3_1080p_s1"]["md5"]
        before = hb.budget()
        assert m2dec_amd.decode_stream_md5(stream("c5_4k_s1"), device=0) == GOLDEN["c5_4k_s1"]["md5"]
        assert m2dec_amd.decode_stream(c3, backend=hb.be) == GOLDEN["c3_1080p_s1"]["md5"]
        after = hb.budget()
    print(before, after)
    for k in ("resident_per_cu", "cap_workgroups", "wg_units", "cap_units", "pics_fit", "streams", "shared"):
        assert before[k] == after[k], (k, before, after)
    assert before["shared"] == 1 and before["cap_workgroups"] > 0 and before["pics_fit"] >= 1


_POOL_SCRIPT = r"""
import sys
sys.path.insert(0, sys.argv[1])
import ctypes, m2dec_amd
from tests._streams import GOLDEN, stream
L = m2dec_amd.lib()
for name in ("c3_1080p_s1", "c5_4k_s1", "c3_1080p_s1"):
    assert m2dec_amd.decode_stream_md5(stream(name), device=0) == GOLDEN[name]["md5"], name
pooled = ctypes.c_longlong()
total = L.m2dec_amd_pinned_bytes(ctypes.byref(pooled))
print("pinned", total, pooled.value, flush=True)
L.m2dec_amd_release_pools()
total2 = L.m2dec_amd_pinned_bytes(ctypes.byref(pooled))
print("released", total2, pooled.value, flush=True)
assert m2dec_amd.decode_stream_md5(stream("c3_1080p_s1"), device=0) == GOLDEN["c3_1080p_s1"]["md5"]
print("ok", flush=True)
"""


@pytest.mark.gpu
def test_gpu_pooled_pinned_bytes_are_capped(built):
    """the parse pool's page-locked job arenas are bounded by M2DEC_AMD_POOL_PINNED_MB, and
    m2dec_amd_release_pools() returns them (the next decode pins anew and is still exact)."""
    import subprocess
    import sys
    env = dict(os.environ, M2DEC_AMD_POOL_PINNED_MB="64")
    r = subprocess.run([sys.executable, "-c", _POOL_SCRIPT, ROOT], env=env, capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = {ln.split()[0]: [int(x) for x in ln.split()[1:]] for ln in r.stdout.splitlines() if ln.strip()}
    total, pooled = lines["pinned"]
    assert 0 < pooled <= 64 << 20, lines
    assert pooled <= total
    assert lines["released"][1] == 0 and lines["released"][0] == 0, lines
    assert "ok" in lines
