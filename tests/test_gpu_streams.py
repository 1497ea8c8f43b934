"""Synthetic streams through the product path (host parser -> HIP back end) on the GPU: every
frame's MD5 must equal the CPU oracle's golden."""
import pytest

import m2dec_amd
from tests._streams import GOLDEN, stream


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_hip_matches_golden(built, name):
    data = stream(name)
    got = m2dec_amd.decode_stream(data)
    want = GOLDEN[name]["md5"]
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert len(got) == len(want) and not bad, f"{name}: frames {bad[:10]} differ (of {len(want)})"


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_hip_batch_replay_matches_golden(built, name):
    """The bench path: every picture of the stream in ONE k_batch launch (slot reuse ordered on the
    device), each picture copied out before its slot is released; MD5s in output order."""
    data = stream(name)
    tr = m2dec_amd.Trace(data)
    rp = m2dec_amd.HipReplay(tr, 0)
    try:
        got = rp.md5_output_order()
    finally:
        rp.close()
        tr.close()
    want = GOLDEN[name]["md5"]
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert len(got) == len(want) and not bad, f"{name}: frames {bad[:10]} differ (of {len(want)})"
