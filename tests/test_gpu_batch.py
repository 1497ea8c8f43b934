"""Several pictures per decode-path launch (runtime.hip be_submit / be_flush, m2r_backend_t.flush): the
pictures parsed in one burst go to the GPU as one k_picture launch, ordered among themselves on the
device.  Bit-exact against the goldens with the default limit, with the most pictures per launch the
budget allows, and with one picture per launch; the launch counters show which one ran."""
import os

import pytest

import m2dec_amd
from tests._streams import GOLDEN, stream

pytestmark = pytest.mark.gpu


def _decode(name, per_launch=None):
    old = os.environ.get("M2DEC_AMD_PICS_PER_LAUNCH")
    try:
        if per_launch is None:
            os.environ.pop("M2DEC_AMD_PICS_PER_LAUNCH", None)
        else:
            os.environ["M2DEC_AMD_PICS_PER_LAUNCH"] = str(per_launch)
        st = m2dec_amd.Stats()
        md5 = m2dec_amd.decode_stream_md5(stream(name), device=0, stats=st)
        return md5, st
    finally:
        if old is None:
            os.environ.pop("M2DEC_AMD_PICS_PER_LAUNCH", None)
        else:
            os.environ["M2DEC_AMD_PICS_PER_LAUNCH"] = old


@pytest.mark.parametrize("name", ["c3_1080p_s1", "cov_cabac_s1", "cov_slices_s1", "cov_wp_s1"])
def test_pictures_per_launch_bit_exact(built, name):
    gold = GOLDEN[name]["md5"]
    one, st1 = _decode(name, 1)
    assert one == gold
    assert st1.kernel_launches == st1.pictures  # one picture per launch
    many, st4 = _decode(name, 4)
    assert many == gold
    assert st4.kernel_launches <= st4.pictures
    dflt, st = _decode(name)
    assert dflt == gold
