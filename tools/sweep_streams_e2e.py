"""8 C4 streams decoded concurrently on one GPU (m2dec_amd_decode_streams_md5) under different
parse-pool / per-stream settings; prints fps per configuration (bit-exact checked)."""
import os
import sys
import resource
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402

names = ["c3_1080p_s1"] + [f"c4_1080p_s{i}" for i in range(2, 9)]
datas = [stream(n) for n in names]
single = datas[0]
for _ in range(2):
    m2dec_amd.decode_stream_md5(single)
t = []
for _ in range(3):
    st = m2dec_amd.Stats()
    assert m2dec_amd.decode_stream_md5(single, stats=st) == GOLDEN[names[0]]["md5"]
    t.append(60 / (st.t_end - st.t_start))
print(f"single stream: {' '.join('%.0f' % x for x in t)} fps", flush=True)
configs = [c.split(":") for c in (sys.argv[1:] or ["3:2", "8:2", "16:2", "16:1"])]
for pt, mt in configs:
    os.environ["M2DEC_AMD_STREAM_PARSE_THREADS"] = pt
    os.environ["M2DEC_AMD_STREAM_MD5_THREADS"] = mt
    res = []
    for _ in range(3):
        r0 = resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        got = m2dec_amd.decode_streams(datas)
        dt = time.perf_counter() - t0
        r1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
        ok = all(g == GOLDEN[n]["md5"] for g, n in zip(got, names))
        res.append((sum(len(g) for g in got) / dt, ok, cpu / dt, (r1.ru_stime - r0.ru_stime) / dt))
    print(f"8 streams, {pt} parse threads / stream, {mt} md5 threads / stream: "
          + " ".join("%.0f%s (%.1f cores, sys %.1f)" % (f, "" if ok else "(BAD)", c, sy) for f, ok, c, sy in res) + " fps",
          flush=True)
