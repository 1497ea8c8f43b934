"""Regenerate tests/golden/synthetic.json: for each synthetic stream (preset, seed, frames) record
the stream's sha256 and the per-frame NV12 MD5s from the CPU oracle (oracle/recon_oracle.c) over
the host parser.  These goldens are oracle-derived ("partially pinned": the oracle itself is pinned
to the reference decoder by the F1 fixture)."""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import m2dec_amd  # noqa: E402
from tests._oracle import OracleBackend  # noqa: E402

GEN = os.path.join(ROOT, "tools", "_build", "h264gen")
STREAMS = [
    # name, preset, seed, frames
    ("cov_cavlc_s1", "cov_cavlc", 1, 16),
    ("cov_cavlc_s2", "cov_cavlc", 2, 16),
    ("cov_cabac_s1", "cov_cabac", 1, 16),
    ("cov_cabac_s2", "cov_cabac", 2, 16),
    ("cov_cabac4x4_s1", "cov_cabac4x4", 1, 16),
    ("cov_wp_s1", "cov_wp", 1, 16),
    ("cov_slices_s1", "cov_slices", 1, 12),
    ("c2_720p_s1", "c2", 1, 60),
    ("c3_1080p_s1", "c3", 1, 60),
    ("c5_4k_s1", "c5", 1, 16),
    # plane prediction, constrained intra (incl. the A#8 no-residual quirk), deblocking idc 2,
    # SPS scaling lists in the reference's layout
    ("cov_tools_s1", "cov_tools", 1, 16),
    ("cov_tools_s2", "cov_tools", 2, 16),
    ("cov_tools_cavlc_s1", "cov_tools_cavlc", 1, 16),
    # explicit weights at the SSE2 int16 saturation and the int8 weight 128 (A#1, A#16), SWAR DC-only
    # adds of 200..255 (A#17): tests/test_quirks.py asserts the oracle's hit counters
    ("cov_wp_quirks_s1", "cov_wp_quirks", 1, 16),
    # reference-picture machinery: list modification idc 0 / 1 / 2, MMCO 1..6, long-term
    # pictures in P / B lists and in temporal direct, IDR long_term_reference_flag, POC types 1 and 2,
    # frame_num wrap, non-reference P pictures; recorded only when the parser's lists and every syntax
    # element equal the generator's (tests/gen_check.py) — tests/test_reflists_cpu.py asserts each path ran
    ("cov_reflists_s1", "cov_reflists", 1, 40),
    ("cov_reflists_s2", "cov_reflists", 2, 40),
    ("cov_reflists_cavlc_s1", "cov_reflists_cavlc", 1, 30),
    ("cov_mmco5_s1", "cov_mmco5", 1, 30),
    ("cov_poc1_s1", "cov_poc1", 1, 24),
    ("cov_poc2_s1", "cov_poc2", 1, 24),
] + [(f"c4_1080p_s{s}", "c3", s, 60) for s in range(2, 9)] \
  + [(f"c5_4k_s{s}", "c5", s, 16) for s in range(2, 9)]  # C4 / C5: one stream per GPU, seed 1 + rank


def gen(preset, seed, frames, out):
    subprocess.run([GEN, "--preset", preset, "--seed", str(seed), "--frames", str(frames), "-o", out], check=True,
                   stderr=subprocess.DEVNULL)
    return open(out, "rb").read()


def main():
    """Only streams missing from the committed file are decoded, unless --all is given."""
    path = os.path.join(ROOT, "tests", "golden", "synthetic.json")
    res = {} if "--all" in sys.argv or not os.path.exists(path) else json.load(open(path))
    tmp = "/tmp/m2dec_goldens"
    os.makedirs(tmp, exist_ok=True)
    for name, preset, seed, frames in STREAMS:
        if name in res:
            continue
        data = gen(preset, seed, frames, os.path.join(tmp, name + ".264"))
        if preset.startswith(("cov_reflists", "cov_mmco5", "cov_poc")):
            from tests import gen_check
            errs = gen_check.check(preset, seed=seed, extra=(f"frames={frames}",), tmpdir=tmp)
            if errs:
                raise SystemExit(f"{name}: parser and generator disagree: {errs[:3]}")
        with OracleBackend() as ob:
            md5s = m2dec_amd.decode_stream(data, backend=ob.be)
        res[name] = {"preset": preset, "seed": seed, "frames": frames, "bytes": len(data),
                     "sha256": hashlib.sha256(data).hexdigest(), "md5": md5s}
        print(name, len(data), len(md5s))
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
