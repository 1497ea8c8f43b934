"""8 C4 streams decoded concurrently on one GPU (m2dec_amd_decode_streams_md5) under different
parse-pool / per-stream settings; prints fps per configuration (bit-exact checked)."""
import os
import sys
import resource
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402

import collections
import threading

TICK = os.sysconf("SC_CLK_TCK")


class ThreadCpu:
    """CPU seconds per thread name (user, sys) over a region, sampled from /proc/self/task every 20 ms
    (threads that exit in between keep their last sample)."""

    def __init__(self):
        self.last = {}
        self.stop = threading.Event()

    def _sample(self):
        for tid in os.listdir("/proc/self/task"):
            try:
                st = open(f"/proc/self/task/{tid}/stat").read()
            except OSError:
                continue
            name = st[st.index("(") + 1:st.rindex(")")]
            f = st[st.rindex(")") + 2:].split()
            self.last[tid] = (name, int(f[11]), int(f[12]))

    def _run(self):
        while not self.stop.is_set():
            self._sample()
            time.sleep(0.02)

    def __enter__(self):
        self._sample()
        self.base = dict(self.last)
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()
        return self

    def __exit__(self, *a):
        self.stop.set()
        self.th.join()
        self._sample()
        acc = collections.defaultdict(lambda: [0.0, 0.0])
        for tid, (name, u, sy) in self.last.items():
            b = self.base.get(tid, (name, 0, 0))
            key = name if name.startswith("m2d-") else ("python" if tid == str(os.getpid()) else "other:" + name[:10])
            acc[key][0] += (u - b[1]) / TICK
            acc[key][1] += (sy - b[2]) / TICK
        self.acc = dict(acc)


names = ["c3_1080p_s1"] + [f"c4_1080p_s{i}" for i in range(2, 9)]
datas = [stream(n) for n in names]
single = datas[0]
for _ in range(2):
    m2dec_amd.decode_stream_md5(single)
t = []
for _ in range(3):
    st = m2dec_amd.Stats()
    r0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    with ThreadCpu() as tc1:
        assert m2dec_amd.decode_stream_md5(single, stats=st) == GOLDEN[names[0]]["md5"]
    dt = time.perf_counter() - t0
    r1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    t.append((60 / (st.t_end - st.t_start), cpu / dt, 1e3 * cpu / 60))
print("single stream: " + " ".join("%.0f fps (%.1f cores, %.1f CPU-ms/frame)" % x for x in t), flush=True)
print("  CPU-ms/frame by thread (user+sys) of the last run: " + ", ".join(
    "%s %.2f+%.2f" % (k, 1e3 * v[0] / 60, 1e3 * v[1] / 60) for k, v in sorted(tc1.acc.items(), key=lambda kv: -sum(kv[1])) if sum(v) > 0.005),
    flush=True)
configs = [c.split(":") for c in (sys.argv[1:] or ["3:2", "8:2", "16:2", "16:1"])]
for pt, mt in configs:
    os.environ["M2DEC_AMD_STREAM_PARSE_THREADS"] = pt
    os.environ["M2DEC_AMD_STREAM_MD5_THREADS"] = mt
    res = []
    for _ in range(3):
        r0 = resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        with ThreadCpu() as tc:
            got = m2dec_amd.decode_streams(datas)
        dt = time.perf_counter() - t0
        r1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
        ok = all(g == GOLDEN[n]["md5"] for g, n in zip(got, names))
        nfr = sum(len(g) for g in got)
        res.append((nfr / dt, ok, cpu / dt, (r1.ru_stime - r0.ru_stime) / dt, 1e3 * cpu / nfr))
    nfr8 = sum(len(g) for g in got)
    print("  CPU-ms/frame by thread (user+sys) of the last pass: " + ", ".join(
        "%s %.2f+%.2f" % (k, 1e3 * v[0] / nfr8, 1e3 * v[1] / nfr8) for k, v in sorted(tc.acc.items(), key=lambda kv: -sum(kv[1])) if sum(v) > 0.005),
        flush=True)
    print(f"8 streams, {pt} parse threads / stream, {mt} md5 threads / stream: "
          + " ".join("%.0f%s (%.1f cores, sys %.1f, %.1f CPU-ms/frame)" % (f, "" if ok else "(BAD)", c, sy, cf) for f, ok, c, sy, cf in res) + " fps",
          flush=True)
