"""Which bench leg slows the C5 (4K, 8 slices) end-to-end decode that runs after it in the same process?
Runs C5 decodes before and after (1) the single-stream replay leg, (2) the 8-stream replay leg, and prints per
block the median decode interval with the per-frame parse CPU, kernel time per launch and setup time, so the
stage that grows is named."""
import os
import statistics
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402


def c5(tag, n=6):
    d = stream("c5_4k_s1")
    rows = []
    for _ in range(n):
        st = m2dec_amd.Stats()
        assert m2dec_amd.decode_stream_md5(d, device=0, stats=st) == GOLDEN["c5_4k_s1"]["md5"]
        rows.append((1e3 * (st.t_end - st.t_start), 1e3 * st.parse_cpu_s / max(1, st.pictures),
                     st.kernel_us / max(1, st.kernel_launches), 1e3 * st.setup_s, st.kernel_launches))
    med = lambda k: statistics.median(r[k] for r in rows)  # noqa: E731
    print(f"{tag:28s} decode median {med(0):7.2f} ms  [{' '.join('%.1f' % r[0] for r in rows)}]  parse/pic "
          f"{med(1):6.2f} ms  kernel/launch {med(2):8.1f} us  setup {med(3):6.2f} ms  launches {med(4):.0f}",
          flush=True)


def replay(names, passes=10):
    traces = [m2dec_amd.Trace(stream(n)) for n in names]
    rp = m2dec_amd.HipReplay(traces if len(traces) > 1 else traces[0], 0)
    rp.md5_output_order()
    t0 = time.perf_counter()
    rp.run(passes)
    rp.sync()
    print(f"replay {len(names)} stream(s): {1e3 * (time.perf_counter() - t0) / passes:.2f} ms per pass", flush=True)
    rp.close()
    for t in traces:
        t.close()


c5("c5 warmup", 2)
c5("c5 fresh")
replay(["c3_1080p_s1"])
c5("c5 after replay x1")
c5("c5 after replay x1 (again)")
replay(["c3_1080p_s1"] + [f"c4_1080p_s{i}" for i in range(2, 9)])
c5("c5 after replay x8")
c5("c5 after replay x8 (again)")
