"""The bench's H.265 leg alone (bench.h265_leg): python tools/h265_bench.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
print(json.dumps(bench.h265_leg(0, steps, 2)), flush=True)
