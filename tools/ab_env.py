"""Interleaved A/B of environment configurations on the c3 end-to-end decode (median decode interval of N
decodes per run, every decode bit-exact).  Usage: python3 tools/ab_env.py ROUNDS N 'NAME:K=V,K=V' ...
(each configuration runs in its own process: GPU_MAX_HW_QUEUES etc. are read when HIP starts).
AB_STREAM=<golden name> picks another stream (default c3_1080p_s1)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, statistics
sys.path.insert(0, os.environ.get('AB_ROOT') or %r)
import m2dec_amd
from tests._streams import stream, GOLDEN
NAME = os.environ.get('AB_STREAM', 'c3_1080p_s1')
d = stream(NAME)
ts = []
def thr():
    try:
        st = dict(l.split() for l in open('/sys/fs/cgroup/cpu.stat'))
        return int(st['nr_throttled']), int(st['throttled_usec']), int(st['nr_periods'])
    except Exception:
        return 0, 0, 0
for i in range(%d + 2):
    if i == 2:
        c0 = thr()
    st = m2dec_amd.Stats()
    md5 = m2dec_amd.decode_stream_md5(d, device=0, stats=st)
    assert md5 == GOLDEN[NAME]['md5']
    if i >= 2:
        ts.append(1e3 * (st.t_end - st.t_start))
c1 = thr()
print('RESULT', statistics.median(ts), min(ts))
print('THROTTLE', c1[0] - c0[0], (c1[1] - c0[1]) / 1e3, c1[2] - c0[2])
print('ALL', ' '.join('%%.3f' %% t for t in ts))
"""


def main():
    rounds, n = int(sys.argv[1]), int(sys.argv[2])
    cfgs = []
    for a in sys.argv[3:]:
        name, _, kv = a.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        cfgs.append((name, env))
    res = {c[0]: [] for c in cfgs}
    every = {c[0]: [] for c in cfgs}
    throttled = {c[0]: [0, 0.0, 0] for c in cfgs}  # CFS periods throttled, ms, periods (cgroup v2 cpu.stat)
    for r in range(rounds):
        for name, env in cfgs:
            e = dict(os.environ, **env)
            out = subprocess.run([sys.executable, "-c", CHILD % (ROOT, n)], env=e, capture_output=True, text=True,
                                 timeout=300)
            line = [x for x in out.stdout.splitlines() if x.startswith("RESULT")]
            if out.returncode or not line:
                print(name, "FAILED", out.returncode, out.stderr[-800:], flush=True)
                sys.exit(1)
            med, mn = map(float, line[0].split()[1:])
            th = [x for x in out.stdout.splitlines() if x.startswith("THROTTLE")]
            thr = th[0].split()[1:] if th else ["?", "?", "?"]
            throttled[name][0] += int(thr[0]) if thr[0] != "?" else 0
            throttled[name][1] += float(thr[1]) if thr[1] != "?" else 0.0
            throttled[name][2] += int(thr[2]) if thr[2] != "?" else 0
            res[name].append(med)
            every[name] += [float(x) for x in [y for y in out.stdout.splitlines() if y.startswith("ALL")][0].split()[1:]]
            print(f"round {r} {name:12s} median {med:6.2f} ms  min {mn:6.2f} ms", flush=True)
    import statistics
    for k, v in every.items():  # every decode of every round: the comparison to read
        v = sorted(v)
        print(f"all {k:12s} n {len(v):3d}  median {statistics.median(v):6.2f}  mean {statistics.mean(v):6.2f}  "
              f"p25 {v[len(v) // 4]:6.2f}  p75 {v[3 * len(v) // 4]:6.2f} ms  throttled {throttled[k][0]} of "
              f"{throttled[k][2]} periods, {throttled[k][1]:.1f} ms", flush=True)
    print(json.dumps({k: sorted(v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
