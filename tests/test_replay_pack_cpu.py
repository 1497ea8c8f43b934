"""Multi-stream replay slot packing (runtime.hip pack_slots), checked on the CPU: each stream of an
interleaved replay gets 64 / n device frame slots, assigned by liveness; every reference of every
picture must still name the content (writer picture) it named in the trace."""
import ctypes

import pytest

import m2dec_amd
from tests._streams import stream


@pytest.mark.parametrize("name,k", [("c3_1080p_s1", 8), ("c3_1080p_s1", 5), ("cov_cabac_s1", 8), ("cov_wp_s1", 6),
                                    ("cov_slices_s1", 8), ("c2_720p_s1", 4)])
def test_pack_preserves_references(built, name, k):
    L = m2dec_amd.lib()
    L.m2dec_amd_replay_pack_check.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.m2dec_amd_replay_pack_check.restype = ctypes.c_int
    t = m2dec_amd.Trace(stream(name))
    try:
        assert t.nslots > k  # the trace names more slots than the packed replay gives the stream
        assert L.m2dec_amd_replay_pack_check(t.h, k) == 0
        assert L.m2dec_amd_replay_pack_check(t.h, 1) == -1  # one slot cannot hold a reference and the picture
    finally:
        t.close()
