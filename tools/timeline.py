"""Line up the host timeline (M2DEC_AMD_TIMELINE, tools/timeline_run.py) with the rocprofv3 kernel / copy trace
of the same run: for the LAST decode, when each picture was parsed, submitted, launched, reconstructed, copied
out and hashed, plus the tail after the last parse.  Usage: python3 tools/timeline.py DIR (tools/timeline.sh)."""
import csv
import glob
import os
import sys

d = sys.argv[1]
host = list(csv.DictReader(open(os.path.join(d, "host.csv"))))
ev = [(int(r["t_ns"]), r["kind"], int(r["a"]), int(r["b"])) for r in host]
ev.sort()
starts = [e for e in ev if e[1] == "D"]
ends = [e for e in ev if e[1] == "d"]
# TL_DECODE=k: the k-th decode of the run (default the last); TL_DECODE=slowest: the longest one
_sel = os.environ.get("TL_DECODE")
TAIL_NS = 100_000 if _sel is not None else 50_000_000  # (a chosen decode: nothing of the next one)
_pairs = list(zip([e[0] for e in starts], [e[0] for e in ends]))
print("decode intervals (ms):", [round((b - a) / 1e6, 2) for a, b in _pairs])
if _sel == "slowest":
    t0, t1 = max(_pairs, key=lambda p: p[1] - p[0])
elif _sel is not None:
    t0, t1 = _pairs[int(_sel)]
else:
    t0, t1 = starts[-1][0], ends[-1][0]
win = [e for e in ev if t0 <= e[0] <= t1 + TAIL_NS]
ms = lambda t: (t - t0) / 1e6  # noqa: E731


def trace(pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


kern = [r for r in trace("*kernel_trace.csv") if int(r["Start_Timestamp"]) >= t0 - 1_000_000 and int(r["End_Timestamp"]) <= t1 + TAIL_NS]
copies = [r for r in trace("*memory_copy_trace.csv") if t0 - 1_000_000 <= int(r["Start_Timestamp"]) <= t1 + TAIL_NS]
print(f"decode interval {ms(t1):.2f} ms  ({len(kern)} kernels, {len(copies)} copies in the window)")

parse = {}
for t, k, a, b in win:
    if k == "P":
        parse[a] = [ms(t), None, b]
    elif k == "p" and a in parse:
        parse[a][1] = ms(t)
sub = {}
for t, k, a, b in win:
    if k == "S":
        sub[a] = [ms(t), None]
    elif k == "s" and a in sub:
        sub[a][1] = ms(t)
disp = {a: (ms(t), b) for t, k, a, b in win if k == "Q"}
colw, cw0 = [], {}
for t, k, a, b in win:
    if k == "W":
        cw0[a] = (ms(t), b)
    elif k == "w" and a in cw0:
        colw.append((a, cw0[a][0], ms(t) - cw0[a][0], cw0[a][1]))
print("\njob  type  dispatch (ahead)  parse start..end    submit")
for s in sorted(parse):
    p = parse[s]
    dq = disp.get(s, (-1, -1))
    print(f"{s:4d}  {p[2]:4d}  {dq[0]:7.2f} ({dq[1]:3d})   {p[0]:7.2f} .. {p[1] if p[1] else -1:7.2f}   {sub.get(s, [-1])[0]:7.2f}")
print("lookahead col-store waits (job, start, ms, until job):", [(a, round(t, 2), round(w, 2), u) for a, t, w, u in colw])

# the serial submission of one picture: acquire (A..a), record copy (a..C), back-end submit (C..s)
acq, cpy, smt = [], [], []
st = {}
for t, k, a, b in win:
    if k in "AaC":
        st[(k, a)] = ms(t)
    elif k == "s" and ("A", a) in st and ("a", a) in st and ("C", a) in st:
        acq.append(st[("a", a)] - st[("A", a)])
        cpy.append(st[("C", a)] - st[("a", a)])
        smt.append(ms(t) - st[("C", a)])
if acq:
    print(f"submission per picture (mean ms): acquire {sum(acq) / len(acq):.3f}  copy {sum(cpy) / len(cpy):.3f}  "
          f"submit {sum(smt) / len(smt):.3f}  (max acquire {max(acq):.3f}, max submit {max(smt):.3f})")
ph = {"waits+H2D": [], "launch_multi": [], "after": []}
lt = None
for t, k, a, b in win:
    if k == "L":
        lt = [ms(t), None, None]
    elif k == "M" and lt:
        lt[1] = ms(t)
    elif k == "N" and lt:
        lt[2] = ms(t)
    elif k == "l" and lt and lt[1] is not None and lt[2] is not None:
        ph["waits+H2D"].append(lt[1] - lt[0])
        ph["launch_multi"].append(lt[2] - lt[1])
        ph["after"].append(ms(t) - lt[2])
        lt = None
if ph["after"]:
    print("launch_held per launch (mean ms):", {k: round(sum(v) / len(v), 3) for k, v in ph.items()},
          "max launch_multi", round(max(ph["launch_multi"]), 3))
launch = [(ms(t), a, b) for t, k, a, b in win if k == "L"]
kp = sorted([r for r in kern if r["Kernel_Name"].startswith("k_picture")], key=lambda r: int(r["Start_Timestamp"]))
print(f"\n{len(launch)} launches (host), {len(kp)} k_picture kernels")
print("launch@host  pics stream | kernel start..end (ms)  dur  pics(grid)")
for i, r in enumerate(kp):
    L = launch[i] if i < len(launch) else (-1, -1, -1)
    g = int(r["Grid_Size_X"]) // 256
    print(f"{L[0]:9.2f}  {L[1]:3d} {L[2]:3d}    | {ms(int(r['Start_Timestamp'])):7.2f} .. {ms(int(r['End_Timestamp'])):7.2f}"
          f"  {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:5.2f}  {g}")
# concurrency of k_picture launches
pts = []
for r in kp:
    pts += [(int(r["Start_Timestamp"]), 1), (int(r["End_Timestamp"]), -1)]
pts.sort()
hist, c, last = {}, 0, pts[0][0] if pts else 0
for t, dd in pts:
    hist[c] = hist.get(c, 0) + t - last
    c += dd
    last = t
print("k_picture concurrency (launches in flight: ms):", {k: round(v / 1e6, 2) for k, v in sorted(hist.items())})
d2h = sorted([r for r in copies if "DEVICE_TO_HOST" in r.get("Direction", r.get("Operation", "")).upper()
              or "D2H" in str(r).upper()], key=lambda r: int(r["Start_Timestamp"]))
print(f"\n{len(d2h)} device->host copies: first {ms(int(d2h[0]['Start_Timestamp'])) if d2h else -1:.2f} last end "
      f"{ms(max(int(r['End_Timestamp']) for r in d2h)) if d2h else -1:.2f} ms")
md5 = [(ms(t), k, a, b) for t, k, a, b in win if k in "Hh"]
print("MD5 batches (start/end, frames, first index):", [(round(t, 2), k, a, b) for t, k, a, b in md5])
outs = [ms(t) for t, k, a, b in win if k == "O"]
syncs = [(ms(t), k, a) for t, k, a, b in win if k in "Yy"]
wait = 0.0
for i in range(0, len(syncs) - 1):
    if syncs[i][1] == "Y" and syncs[i + 1][1] == "y":
        wait += syncs[i + 1][0] - syncs[i][0]
print(f"frames out: first {outs[0] if outs else -1:.2f} last {outs[-1] if outs else -1:.2f} ms; API thread in sync_frame waits {wait:.2f} ms")
lp = max(p[1] for p in parse.values() if p[1])
lk = max(ms(int(r["End_Timestamp"])) for r in kp) if kp else -1
print(f"\nlast parse end {lp:.2f} | last k_picture end {lk:.2f} (+{lk - lp:.2f}) | last D2H end "
      f"{ms(max(int(r['End_Timestamp']) for r in d2h)) if d2h else -1:.2f} | last frame out {outs[-1] if outs else -1:.2f} | "
      f"last MD5 end {max([t for t, k, a, b in md5 if k == 'h'], default=-1):.2f} | decode end {ms(t1):.2f}")
