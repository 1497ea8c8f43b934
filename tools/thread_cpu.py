"""CPU seconds per thread name over timed 8-stream passes (or c3 decodes): python3 tools/thread_cpu.py
[streams|c3] [passes] — the library names its threads (m2d-parse, m2d-md5, m2d-copy, m2d-stream, m2d-reaper,
m2d-h265); the HIP runtime's and Python's show under their own names.  Reads /proc/self/task/*/stat."""
import collections
import os
import sys
import time

sys.path.insert(0, os.environ.get("AB_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402

TCK = os.sysconf("SC_CLK_TCK")


def snap():
    out = {}
    for t in os.listdir("/proc/self/task"):
        try:
            name = open(f"/proc/self/task/{t}/comm").read().strip()
            if int(t) == os.getpid():
                name += " (main)"  # the caller's thread: the decoder's API / lookahead side; the others of that
                # name are the HIP runtime's
            f = open(f"/proc/self/task/{t}/stat").read().rsplit(")", 1)[1].split()
            out[t] = (name, (int(f[11]) + int(f[12])) / TCK)
        except OSError:
            pass
    return out


mode = sys.argv[1] if len(sys.argv) > 1 else "streams"
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
names = ["c3_1080p_s1"] + [f"c4_1080p_s{i}" for i in range(2, 9)]
datas = [stream(n) for n in (names if mode == "streams" else names[:1])]


def run():
    if mode == "streams":
        got = m2dec_amd.decode_streams(datas)
        assert all(g == GOLDEN[n]["md5"] for g, n in zip(got, names))
        return sum(len(g) for g in got)
    md5 = m2dec_amd.decode_stream_md5(datas[0], device=0)
    assert md5 == GOLDEN["c3_1080p_s1"]["md5"]
    return len(md5)


run()
run()
# threads that end inside the timed passes (each pass's m2d-stream / m2d-md5 threads) are gone from
# /proc/self/task: with M2DEC_AMD_THREAD_CPU=1 the library prints their CPU time on stderr as they end
exited = os.environ.get("M2DEC_AMD_THREAD_CPU") == "1"
if exited:
    sys.stderr.flush()
    log = open("/tmp/thread_cpu_%d.log" % os.getpid(), "w+")
    saved = os.dup(2)
    os.dup2(log.fileno(), 2)
a = snap()
t0, fr = time.perf_counter(), 0
r0 = os.times()
for _ in range(passes):
    fr += run()
dt = time.perf_counter() - t0
r1 = os.times()
b = snap()
by = collections.defaultdict(float)
nth = collections.Counter()
for t, (name, cpu) in b.items():
    by[name] += cpu - a.get(t, (name, 0.0))[1]
    nth[name] += 1
if exited:
    os.dup2(saved, 2)
    log.seek(0)
    for line in log:
        f = line.split()
        if len(f) == 3 and f[0] == "thread-cpu":
            by[f[1] + " (exited)"] += float(f[2]) / 1e3
            nth[f[1] + " (exited)"] += 1
proc = (r1.user - r0.user) + (r1.system - r0.system)
print(f"{mode}: {fr / dt:.1f} fps, {proc / dt:.2f} cores busy ({(r1.system - r0.system) / dt:.2f} system), "
      f"{1e3 * proc / fr:.2f} CPU-ms per frame")
for name, cpu in sorted(by.items(), key=lambda kv: -kv[1]):
    if cpu > 0:
        print(f"  {name:18s} {nth[name]:3d} threads {cpu:7.3f} s  {1e3 * cpu / fr:6.3f} CPU-ms per frame")
