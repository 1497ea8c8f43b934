"""MPEG-1/2 pictures reconstructed on gfx950 (m2dec_amd/csrc/hip/m2v_hip.hip, m2dec_amd_m2v_use_gpu):
every stream of tests/golden/m2v.json — intra (C1 and the coverage streams) and P / B (frame / field /
dual-prime MC, skips, lost slices, MPEG-1) — must give the golden MD5 of every frame, the goldens being
the product's host decode checked frame by frame against the oracle's restatement of the reference
(tools/make_m2v_goldens.py)."""
import pytest

import m2dec_amd
from tests.test_mpeg2_cpu import GOLD, m2v_stream

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(GOLD))
def test_gpu_m2v_matches_golden(built, name):
    assert m2dec_amd.decode_m2v(m2v_stream(name), device=0) == GOLD[name]["md5"]


def test_gpu_m2v_emptify(built):
    data = m2v_stream("c1_pb_480p_s1")
    assert m2dec_amd.decode_m2v(data, device=0, emptify=True) == GOLD["c1_pb_480p_s1"]["md5"]
