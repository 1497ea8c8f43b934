"""Bisect a full-speed mismatch: decode streams under debug knobs (see runtime.hip dbg_knob)."""
import os, sys, faulthandler
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.dump_traceback_later(240, exit=True)
import m2dec_amd
from tests._streams import GOLDEN, stream

names = sys.argv[1:] or ["cov_cabac4x4_s1", "cov_slices_s1", "cov_wp_s1", "c2_720p_s1"]
knobs = [{}, {"M2DEC_AMD_SYNC": "1"}, {"M2DEC_AMD_RAW": "1"}, {"M2DEC_AMD_SER": "1"}, {"M2DEC_AMD_RAW": "1", "M2DEC_AMD_SER": "1"}]
for kn in knobs:
    for k in ("M2DEC_AMD_SYNC", "M2DEC_AMD_RAW", "M2DEC_AMD_SER"):
        os.environ.pop(k, None)
    os.environ.update(kn)
    res = []
    for n in names:
        got = m2dec_amd.decode_stream(stream(n))
        want = GOLDEN[n]["md5"]
        bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
        res.append(f"{n}:{len(bad)}/{len(want)}")
    print(kn, " ".join(res), flush=True)
