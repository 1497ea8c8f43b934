"""Interleaved A/B of environment configurations on the 8-stream end-to-end leg (bench.py
end_to_end_streams: the C4 streams decoded concurrently on one GPU, one host thread and decoder context
each, every frame checked).  Each configuration runs in its own process (GPU_MAX_HW_QUEUES etc. are read
when HIP starts); per pass: aggregate fps, host cores busy, system-time cores.
Usage: python3 tools/ab_streams.py ROUNDS PASSES 'NAME:K=V,K=V' ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, time, resource
sys.path.insert(0, os.environ.get('AB_ROOT') or %r)
import m2dec_amd
from tests._streams import stream, GOLDEN
names = ["c3_1080p_s1"] + ["c4_1080p_s%%d" %% i for i in range(2, 9)]
datas = [stream(n) for n in names]
got = m2dec_amd.decode_streams(datas)  # warmup pass
assert all(g == GOLDEN[n]["md5"] for g, n in zip(got, names))
for _ in range(%d):
    r0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    got = m2dec_amd.decode_streams(datas)
    dt = time.perf_counter() - t0
    r1 = resource.getrusage(resource.RUSAGE_SELF)
    assert all(g == GOLDEN[n]["md5"] for g, n in zip(got, names))
    nfr = sum(len(g) for g in got)
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    print("PASS %%.1f %%.2f %%.2f" %% (nfr / dt, cpu / dt, (r1.ru_stime - r0.ru_stime) / dt), flush=True)
"""


def main():
    rounds, passes = int(sys.argv[1]), int(sys.argv[2])
    cfgs = []
    for a in sys.argv[3:]:
        name, _, kv = a.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        cfgs.append((name, env))
    res = {n: [] for n, _ in cfgs}
    for r in range(rounds):
        for name, env in cfgs:
            e = dict(os.environ)
            e.update(env)
            p = subprocess.run([sys.executable, "-c", CHILD % (ROOT, passes)], env=e, capture_output=True, text=True,
                               timeout=300)
            if p.returncode != 0:
                print(f"round {r} {name}: FAILED\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            rows = [tuple(float(v) for v in l.split()[1:]) for l in p.stdout.splitlines() if l.startswith("PASS")]
            res[name] += rows
            print(f"round {r} {name:12s} " + "  ".join("%.0f fps %.1f cores sys %.1f" % x for x in rows), flush=True)
    for name, _ in cfgs:
        f = sorted(x[0] for x in res[name])
        c = sorted(x[1] for x in res[name])
        print(f"all {name:12s} n {len(f):3d}  median {f[len(f) // 2]:7.1f} fps  max {f[-1]:7.1f}  cores {c[len(c) // 2]:.1f}",
              flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
