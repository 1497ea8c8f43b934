"""Medians of an H.265 A/B file written by tools/gpu_run.sh h265ab (lines: VAR=V {json of tools/h265_bench.py})."""
import json
import statistics
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for line in open(sys.argv[1]):
    cfg, _, js = line.partition(" ")
    for name, leg in json.loads(js).items():
        vals[name][cfg].append(leg["value"])
for name, by in vals.items():
    for cfg, v in by.items():
        print(f"{name:24s} {cfg:28s} n {len(v)}  median {statistics.median(v):8.2f} fps  all {v}")
