"""c2/c3 deterministic mismatch: replay (serial, per-picture) vs golden, and the backend with SYNC."""
import os, sys, faulthandler
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.enable()
faulthandler.dump_traceback_later(200, exit=True)
import m2dec_amd
from tests._streams import GOLDEN, stream
for n in sys.argv[1:]:
    data = stream(n)
    want = GOLDEN[n]["md5"]
    tr = m2dec_amd.Trace(data)
    print(n, "trace", tr.npics, tr.width, tr.height, flush=True)
    os.environ["M2DEC_AMD_DEBUG"] = "1"
    rp = m2dec_amd.HipReplay(tr, 0)
    md = rp.md5_output_order()
    os.environ.pop("M2DEC_AMD_DEBUG")
    print(n, "replay serial bad:", [i for i, (a, b) in enumerate(zip(md, want)) if a != b][:20], flush=True)
    os.environ["M2DEC_AMD_SYNC"] = "1"
    got = m2dec_amd.decode_stream(data)
    os.environ.pop("M2DEC_AMD_SYNC")
    print(n, "decode SYNC bad:", [i for i, (a, b) in enumerate(zip(got, want)) if a != b][:20], flush=True)
