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
