"""The bench's H.265 legs alone (bench.h265_leg): python tools/h265_bench.py [steps] [golden name ...]
(default: the intra and the P / B 1080p streams)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
names = sys.argv[2:] or ["c_h265_1080p_s1", "c_h265_1080p_pb_s1"]
print(json.dumps({n: bench.h265_leg(0, steps, 2, n) for n in names}), flush=True)
