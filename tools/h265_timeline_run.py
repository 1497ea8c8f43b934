"""H.265 decodes for a timeline: python3 tools/h265_timeline_run.py NAME N — each decode through the GPU back end
(bench.h265_leg's path) with M2DEC_AMD_H265_TRACE set (the parse jobs' start / end / submit on stderr) and the
decode's own bracket on stdout, all on CLOCK_MONOTONIC like rocprofv3's timestamps (tools/h265_timeline.sh)."""
import json
import os
import sys
import time

os.environ["M2DEC_AMD_H265_TRACE"] = "1"
if len(sys.argv) > 3:  # the host event timeline (timeline.c: frames out, MD5 batches, sync_frame) to this CSV
    os.environ["M2DEC_AMD_TIMELINE"] = sys.argv[3]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import m2dec_amd  # noqa: E402
from test_h265_cpu import h265_stream  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c_h265_1080p_pb_s1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
g = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "h265.json")))[name]
data = h265_stream(name)
with m2dec_amd.H265HipBackend(0) as be:
    for i in range(n):
        sys.stderr.write("decode %d begin %.3f\n" % (i, time.monotonic() * 1e3))
        t0 = time.monotonic()
        md5, _ = m2dec_amd.decode_h265_md5(data, backend=be.be)
        t1 = time.monotonic()
        sys.stderr.write("decode %d end %.3f\n" % (i, t1 * 1e3))
        print("decode", i, "ok", md5 == g["md5"], "%.2f ms" % ((t1 - t0) * 1e3), flush=True)
