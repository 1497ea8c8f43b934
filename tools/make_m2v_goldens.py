"""Regenerate tests/golden/m2v.json: for each synthetic MPEG-1/2 stream (tools/_build/m2vgen preset,
seed, frames) the stream's sha256 and the per-frame MD5 lines of `h264dec -O`, decoded by the product
(m2d_func) AND by the pure-Python restatement oracle/mpeg2_oracle.py (which reads the reference's own
VLC tables from tests/golden/mpeg2_vlc.json); a stream is only recorded when both agree on every frame.
Whole streams stay "parity unpinned" (no reference-produced output exists for them)."""
import ctypes
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import m2dec_amd  # noqa: E402
import mpeg2_oracle  # noqa: E402

GEN = os.path.join(ROOT, "tools", "_build", "m2vgen")
STREAMS = [("c1_480p_s1", "c1", 1, 30), ("cov_m2v_s1", "cov_m2v", 1, 8), ("cov_m2v_s2", "cov_m2v", 2, 8),
           ("cov_m2v_slices_s1", "cov_m2v_slices", 1, 8), ("cov_mpeg1_s1", "cov_mpeg1", 1, 6),
           # P / B pictures (coded order I P B B ...): frame / field / dual-prime MC, skips, lost slices
           ("c1_pb_480p_s1", "c1_pb", 1, 30), ("cov_m2v_pb_s1", "cov_m2v_pb", 1, 10),
           ("cov_m2v_pb_s2", "cov_m2v_pb", 2, 10), ("cov_m2v_pb_field_s1", "cov_m2v_pb_field", 1, 10),
           ("cov_m2v_pb_field_s2", "cov_m2v_pb_field", 2, 10), ("cov_mpeg1_pb_s1", "cov_mpeg1_pb", 1, 10)]


def gen(preset, seed, frames):
    out = f"/tmp/m2v_gold_{os.getpid()}.m2v"
    subprocess.run([GEN, "--preset", preset, "--seed", str(seed), "--frames", str(frames), "-o", out], check=True)
    data = open(out, "rb").read()
    os.unlink(out)
    return data


def main():
    path = os.path.join(ROOT, "tests", "golden", "m2v.json")
    res = {}
    for name, preset, seed, frames in STREAMS:
        data = gen(preset, seed, frames)
        got = m2dec_amd.decode_m2v(data)
        assert m2dec_amd.m2v_last_checks() == (0, 0), f"{name}: output depends on reference UB"
        ref = mpeg2_oracle.decode(data)
        assert got == ref, f"{name}: product and oracle differ on frames " \
                           f"{[i for i, (a, b) in enumerate(zip(got, ref)) if a != b][:8]} ({len(got)} vs {len(ref)})"
        res[name] = {"preset": preset, "seed": seed, "frames": frames, "bytes": len(data),
                     "sha256": hashlib.sha256(data).hexdigest(), "md5": got}
        print(name, len(data), len(got))
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
