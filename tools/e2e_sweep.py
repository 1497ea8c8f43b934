"""End-to-end single-stream decode (h264d_func + MD5 helper threads, like h264dec -O) of the C3 stream:
frames/s for a grid of parse-ahead workers x MD5 threads, every run checked against the golden MD5s.
Usage: python tools/e2e_sweep.py [preset_name] ; env M2DEC_AMD_ASYNC_STATS=1 prints the pipeline split."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3_1080p_s1"
data = stream(name)
print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)), flush=True)
m2dec_amd.decode_stream_md5(data)  # warm: device init, page-in
for pt in (8, 12, 16):
    for mt in (4, 8):
        os.environ["M2DEC_AMD_PARSE_THREADS"] = str(pt)
        os.environ["M2DEC_AMD_MD5_THREADS"] = str(mt)
        best = 0.0
        for _ in range(3):
            t0 = time.perf_counter()
            got = m2dec_amd.decode_stream_md5(data)
            dt = time.perf_counter() - t0
            assert got == GOLDEN[name]["md5"], "not bit-exact"
            best = max(best, len(got) / dt)
        print(f"parse {pt:2d} md5 {mt:2d}: {best:7.1f} fps", flush=True)
