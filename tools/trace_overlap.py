"""Overlap of the decode path's k_picture launches in a rocprofv3 kernel trace: per 60-picture step,
the span, the summed launch durations (their ratio = pictures in flight on average) and the gaps.
Usage: python tools/trace_overlap.py gpurun_out/prof_TAG/run_kernel_trace.csv"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith("k_picture")]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
seg = [[ev[0]]]
for e in ev[1:]:
    if e[0] - max(x[1] for x in seg[-1]) > 3e6:
        seg.append([e])
    else:
        seg[-1].append(e)
for s in seg:
    if len(s) < 30:
        continue
    t0 = s[0][0]
    span = max(x[1] for x in s) - t0
    busy = sum(x[1] - x[0] for x in s)
    idle, end = 0, s[0][1]
    for a, b in s[1:]:
        if a > end:
            idle += a - end
        end = max(end, b)
    print(f"pictures {len(s)}  span {span / 1e6:.2f} ms  sum {busy / 1e6:.2f} ms  in flight {busy / span:.2f}  "
          f"device idle {idle / 1e6:.2f} ms  mean launch {busy / len(s) / 1e3:.0f} us")
