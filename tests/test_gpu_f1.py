"""F1 through the product path (host parser -> HIP gfx950 back end), vs the reference MD5s."""
import os

import pytest

import m2dec_amd
from tests._oracle import golden_md5s, ROOT

GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.mark.gpu
def test_f1_hip_matches_reference(built):
    assert m2dec_amd.hip_available(), "no gfx950 device visible"
    data = open(os.path.join(GOLD, "f1_realshort.264"), "rb").read()
    got = m2dec_amd.decode_stream(data)
    want = golden_md5s(os.path.join(GOLD, "f1_realshort.md5"))
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert len(got) == len(want) and not bad, f"mismatching frames {bad[:10]} of {len(want)}"


@pytest.mark.gpu
def test_f1_hip_batch_replay_matches_reference(built):
    """F1 parsed once, then reconstructed by ONE k_batch launch (the bench path)."""
    data = open(os.path.join(GOLD, "f1_realshort.264"), "rb").read()
    tr = m2dec_amd.Trace(data)
    rp = m2dec_amd.HipReplay(tr, 0)
    try:
        got = rp.md5_output_order()
    finally:
        rp.close()
        tr.close()
    want = golden_md5s(os.path.join(GOLD, "f1_realshort.md5"))
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert len(got) == len(want) and not bad, f"mismatching frames {bad[:10]} of {len(want)}"
