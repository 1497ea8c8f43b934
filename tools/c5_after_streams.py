"""Does the C5 (4K, 8 slices) end-to-end decode slow down after the 8-stream leg in the same process (as in
bench.py's order)?  Prints the median decode interval of C5 before and after eight concurrent c3/c4 streams."""
import os
import statistics
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402


def c5(n):
    d = stream("c5_4k_s1")
    ts = []
    for _ in range(n):
        st = m2dec_amd.Stats()
        assert m2dec_amd.decode_stream_md5(d, device=0, stats=st) == GOLDEN["c5_4k_s1"]["md5"]
        ts.append(1e3 * (st.t_end - st.t_start))
    return ts


c5(2)
a = c5(6)
print("c5 before: median %.2f ms  %s" % (statistics.median(a), " ".join("%.1f" % x for x in a)), flush=True)
names = ["c3_1080p_s1"] + [f"c4_1080p_s{i}" for i in range(2, 9)]
datas = [stream(n) for n in names]
for _ in range(3):
    t0 = time.perf_counter()
    got = m2dec_amd.decode_streams(datas)
    assert all(g == GOLDEN[n]["md5"] for g, n in zip(got, names))
    print("8 streams pass %.1f ms" % (1e3 * (time.perf_counter() - t0)), flush=True)
b = c5(8)
print("c5 after: median %.2f ms  %s" % (statistics.median(b), " ".join("%.1f" % x for x in b)), flush=True)
