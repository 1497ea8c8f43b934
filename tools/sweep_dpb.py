"""Single-stream decode path (h264dec -O -d n): frames/s and parity per DPB size."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402
data = stream("c3_1080p_s1")
for dpb in [int(x) for x in sys.argv[1:]] or [-1, 4, 8, 16]:
    m2dec_amd.decode_stream_md5(data, dpb=dpb)
    fps = []
    for _ in range(3):
        t0 = time.perf_counter()
        got = m2dec_amd.decode_stream_md5(data, dpb=dpb)
        fps.append(round(len(got) / (time.perf_counter() - t0), 1))
    print("dpb", dpb, fps, "fps", "bit-exact" if got == GOLDEN["c3_1080p_s1"]["md5"] else "MISMATCH", flush=True)
