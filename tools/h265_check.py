"""Decode H.265 goldens on the GPU and report per stream: python3 tools/h265_check.py [name ...]
(environment knobs such as M2DEC_AMD_H265_WAVES apply); prints ok / WRONG (first differing picture) / error."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import m2dec_amd  # noqa: E402
from test_h265_cpu import h265_stream  # noqa: E402

GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "h265.json")))
bad = 0
for name in sys.argv[1:] or sorted(GOLD):
    t0 = time.time()
    md5s, err = m2dec_amd.decode_h265(h265_stream(name), device=0)
    want = GOLD[name]["md5"]
    diff = [i for i, (a, b) in enumerate(zip(md5s, want)) if a != b]
    ok = err == -2 and md5s == want
    bad += not ok
    print(f"{name:28s} {'ok' if ok else 'WRONG'} err={err} pictures {len(md5s)}/{len(want)} first diff {diff[:1]} "
          f"{time.time() - t0:.2f} s", flush=True)
sys.exit(1 if bad else 0)
