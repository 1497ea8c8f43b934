"""C5 after each bench leg, in bench.py's order (main c3 leg, single replay, 8 concurrent streams, 8-stream
replay), to find which leg leaves the process in a state that slows the C5 (4K, 8 slices) decode.  Prints per
block the median decode interval, pictures per launch and the decode contexts the budget sees."""
import ctypes
import os
import statistics
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402

C5 = stream("c5_4k_s1")
NAMES = ["c3_1080p_s1"] + [f"c4_1080p_s{i}" for i in range(2, 9)]


def c5(tag, n=5):
    rows = []
    for _ in range(n):
        st = m2dec_amd.Stats()
        assert m2dec_amd.decode_stream_md5(C5, device=0, stats=st) == GOLDEN["c5_4k_s1"]["md5"]
        rows.append((1e3 * (st.t_end - st.t_start), st.pictures / max(1, st.kernel_launches),
                     1e3 * st.parse_cpu_s / max(1, st.pictures), st.kernel_us / max(1, st.kernel_launches),
                     st.h2d_us / max(1, st.pictures), st.d2h_us / max(1, st.pictures), 1e3 * st.setup_s))
    print(f"{tag:34s} c5 median {statistics.median(r[0] for r in rows):7.2f} ms [{' '.join('%.1f' % r[0] for r in rows)}] "
          f"pics/launch {statistics.median(r[1] for r in rows):.2f} parse/pic {statistics.median(r[2] for r in rows):.2f} ms "
          f"kernel/launch {statistics.median(r[3] for r in rows):.0f} us h2d/pic {statistics.median(r[4] for r in rows):.0f} us "
          f"d2h/pic {statistics.median(r[5] for r in rows):.0f} us setup {statistics.median(r[6] for r in rows):.1f} ms",
          flush=True)


def replay(names, passes=5):
    traces = [m2dec_amd.Trace(stream(n)) for n in names]
    rp = m2dec_amd.HipReplay(traces if len(traces) > 1 else traces[0], 0)
    rp.md5_output_order()
    rp.run(passes)
    rp.sync()
    rp.close()
    for t in traces:
        t.close()


LATE = os.environ.get("C5_LATE") == "1"  # bench.py's order: no C5 before the 1080p legs
if not LATE:
    c5("warm", 2)
    c5("fresh")
c3 = stream("c3_1080p_s1")
for _ in range(25):
    assert m2dec_amd.decode_stream_md5(c3, device=0) == GOLDEN["c3_1080p_s1"]["md5"]
if not LATE:
    c5("after main leg (25 c3 decodes)")
replay(["c3_1080p_s1"])
if not LATE:
    c5("after single replay")
datas = [stream(n) for n in NAMES]
for _ in range(5):
    t0 = time.perf_counter()
    got = m2dec_amd.decode_streams(datas)
    assert all(g == GOLDEN[n]["md5"] for g, n in zip(got, NAMES))
print("8-stream pass %.1f ms" % (1e3 * (time.perf_counter() - t0)), flush=True)
if not LATE:
    c5("after 8 concurrent streams")
replay(NAMES)
if os.environ.get("C5_RELEASE") == "1":  # every pooled job / arena / device buffer freed first
    m2dec_amd.lib().m2dec_amd_release_pools()
if LATE:
    c5("first C5 (2 decodes)", 2)
    pooled = ctypes.c_longlong(0)
    total = m2dec_amd.lib().m2dec_amd_pinned_bytes(ctypes.byref(pooled))
    print("pinned MB %.0f pooled %.0f" % (total / 1e6, pooled.value / 1e6), flush=True)
c5("after 8-stream replay")
c5("again")
