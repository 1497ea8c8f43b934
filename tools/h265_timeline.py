"""Line up the H.265 parse jobs (M2DEC_AMD_H265_TRACE) with the rocprofv3 kernel trace of the same run, for the
LAST decode: python3 tools/h265_timeline.py DIR (tools/h265_timeline.sh)."""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
jobs, dec = {}, {}
for line in open(os.path.join(d, "trace.err")):
    m = re.match(r"h265 job (\d+) (start|end|submit|submitted) ([\d.]+)", line)
    if m:
        jobs.setdefault(int(m.group(1)), {})[m.group(2)] = float(m.group(3))
    m = re.match(r"decode (\d+) (begin|end) ([\d.]+)", line)
    if m:
        dec.setdefault(int(m.group(1)), {})[m.group(2)] = float(m.group(3))
last = max(dec)
t0, t1 = dec[last]["begin"], dec[last]["end"]
print(f"decode {last}: {t1 - t0:.2f} ms")
print("job   parse start .. end  (ms)   submit .. done")
for s in sorted(jobs):
    j = jobs[s]
    if not (t0 <= j.get("start", 0) <= t1):
        continue
    print(f"{s:4d}  {j['start'] - t0:7.2f} .. {j['end'] - t0:7.2f} ({j['end'] - j['start']:6.2f})   "
          f"{j.get('submit', 0) - t0:7.2f} .. {j.get('submitted', 0) - t0:7.2f}")
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
kern = []
for r in (csv.DictReader(open(f[0])) if f else []):
    a, b = int(r["Start_Timestamp"]) / 1e6, int(r["End_Timestamp"]) / 1e6
    if t0 - 1 <= a <= t1 + 1:
        nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        kern.append((a - t0, b - t0, nm, r.get("Queue_Id", r.get("Stream_Id", "?"))))
print("\nkernel                      queue   start ..   end   (us)")
for a, b, nm, q in sorted(kern):
    print(f"{nm:26s} {q:>6s} {a:7.2f} .. {b:7.2f} ({(b - a) * 1e3:7.1f})")

# host events (timeline.c) of the same decode: frames handed to the writer (O), sync_frame (Y/y), MD5 batches (H/h)
tl = os.path.join(d, "host_tl.csv")
if os.path.exists(tl):
    ev = []
    for r in csv.DictReader(open(tl)):
        t = int(r["t_ns"]) / 1e6
        if t0 <= t <= t1:
            ev.append((t - t0, r["kind"], int(r["a"]), int(r["b"])))
    ev.sort()
    print("\nhost events (ms): O frame out (a = index), Y/y sync_frame (a = slot), H/h MD5 batch (a = frames, b = first)")
    print("  " + "  ".join(f"{k}{a}/{b}@{t:.2f}" for t, k, a, b in ev if k in "OYyHh"))
