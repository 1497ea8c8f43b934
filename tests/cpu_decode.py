"""CPU baseline for bench.py (test infrastructure: the oracle is the checker, timed here only as the
CPU leg): the full CPU decode of a synthetic stream — this repo's host parser (CABAC/CAVLC, MV, DPB)
on the caller's thread + the CPU restatement of the reconstruction (oracle/recon_oracle.c) + the
FileWriterMd5 line per frame — through the same h264d_func loop as `h264dec -O`, on one core.

    python -m tests.cpu_decode PRESET SEED FRAMES [STREAMS]

STREAMS > 1 runs that many independent decodes at once, one process each (the all-cores form).
Prints one JSON line: frames, seconds (wall of the slowest process), bit-exactness vs the golden.
"""
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _one(args):
    preset, seed, frames = args
    import m2dec_amd
    from tests._oracle import OracleBackend
    from tests._streams import GOLDEN, stream

    name = {"c3": "c3_1080p_s1" if seed == 1 else f"c4_1080p_s{seed}", "c2": f"c2_720p_s{seed}",
            "c5": f"c5_4k_s{seed}"}[preset]
    g = GOLDEN.get(name)
    if g is None or g["frames"] != frames:
        raise SystemExit(f"cpu_decode: no golden for {name} at {frames} frames")
    data = stream(name)
    with OracleBackend() as ob:
        t0 = time.perf_counter()
        md5 = m2dec_amd.decode_stream(data, backend=ob.be, parse_threads=0)
        dt = time.perf_counter() - t0
    return len(md5), dt, md5 == g["md5"]


def main():
    preset, seed, frames = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    if n == 1:
        res = [_one((preset, seed, frames))]
    else:
        with mp.get_context("spawn").Pool(n) as p:
            res = p.map(_one, [(preset, seed, frames)] * n)
    print(json.dumps({"frames": sum(r[0] for r in res), "seconds": max(r[1] for r in res),
                      "bit_exact": all(r[2] for r in res), "streams": n}), flush=True)


if __name__ == "__main__":
    main()
