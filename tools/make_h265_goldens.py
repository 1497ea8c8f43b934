#!/usr/bin/env python3
"""Make tests/golden/h265.json: for each synthetic H.265 stream (tools/h265gen), the stream's sha256 and
the MD5 line of every output frame, decoded through h265d_func with the CPU oracle's reconstruction
(oracle/h265_oracle.c).  A stream is recorded only when
  * the parser's syntax (CU modes, every residual level) equals the generator's own dump, and
  * the oracle saw no CLIP255C argument outside the reference table's domain and no DC-only term the
    reference's byte-wise SWAR add would corrupt (reference undefined / quirky behaviour).
Parity is "unpinned": no reference-produced H.265 output exists here (the reference is unbuildable,
DESIGN.md §4) and the generator is this repository's own.
Run: python3 tools/make_h265_goldens.py   (after `make`)"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import m2dec_amd  # noqa: E402
import _oracle  # noqa: E402

GEN = os.path.join(ROOT, "tools", "_build", "h265gen")
STREAMS = [("cov_h265_a_s1", "cov_h265_a", 1, 3), ("cov_h265_a_s2", "cov_h265_a", 2, 3),
           ("cov_h265_b_s1", "cov_h265_b", 1, 3), ("cov_h265_b_s2", "cov_h265_b", 2, 3),
           ("cov_h265_c_s2", "cov_h265_c", 2, 3), ("cov_h265_c_s3", "cov_h265_c", 3, 3),
           ("cov_h265_nodbk_s1", "cov_h265_nodbk", 1, 2), ("cov_h265_nosao_s1", "cov_h265_nosao", 1, 2),
           ("cov_h265_hiqp_s1", "cov_h265_hiqp", 1, 2), ("cov_h265_a_long_s3", "cov_h265_a", 3, 20),
           ("c_h265_1080p_s1", "c_h265_1080p", 1, 8),
           # P / B pictures: merge / AMVP / TMVP, bi-prediction, AMP, inter transform trees, inter deblocking
           ("cov_h265_p_s1", "cov_h265_p", 1, 6), ("cov_h265_p_s2", "cov_h265_p", 2, 6),
           ("cov_h265_hb_s1", "cov_h265_hb", 1, 8), ("cov_h265_hb_s2", "cov_h265_hb", 2, 8),
           ("cov_h265_ldb_s1", "cov_h265_ldb", 1, 8), ("cov_h265_ldb_s2", "cov_h265_ldb", 2, 8),
           ("cov_h265_pnodbk_s1", "cov_h265_pnodbk", 1, 5), ("c_h265_1080p_pb_s1", "c_h265_1080p_pb", 1, 8)]


def gen(preset, seed, frames, dump=None):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "s.265")
        cmd = [GEN, "--preset", preset, "--seed", str(seed), "--frames", str(frames), "-o", out]
        if dump:
            cmd += ["--dump", dump]
        subprocess.run(cmd, check=True)
        return open(out, "rb").read()


def check_syntax(preset, seed, frames):
    """(generator dump, decoder dump) equal?"""
    with tempfile.TemporaryDirectory() as d:
        g, p = os.path.join(d, "gen.txt"), os.path.join(d, "dec.txt")
        data = gen(preset, seed, frames, g)
        m2dec_amd.lib().m2dec_amd_h265_set_dump(p.encode())
        try:
            with _oracle.Oracle265Backend() as o:
                m2dec_amd.decode_h265(data, backend=o.be)
        finally:
            m2dec_amd.lib().m2dec_amd_h265_set_dump(None)
        a, b = open(g).read().splitlines(), open(p).read().splitlines()
        return a == [line for line in b if line.startswith(("pic", "cu", "res", "icu", "pu"))], len(a), b


def main():
    out = {}
    for name, preset, seed, frames in STREAMS:
        data = gen(preset, seed, frames)
        ok, nlines, _ = check_syntax(preset, seed, frames)
        _oracle.h265_violations(True)
        with _oracle.Oracle265Backend() as o:
            md5s, err = m2dec_amd.decode_h265(data, backend=o.be)
        viol = _oracle.h265_violations(True)
        print(f"{name}: {len(md5s)} frames, syntax {'==' if ok else '!='} generator ({nlines} lines), violations {viol}")
        if not ok or viol or err != -2 or not md5s:
            print("  not recorded")
            continue
        out[name] = {"preset": preset, "seed": seed, "frames": frames, "sha256": hashlib.sha256(data).hexdigest(),
                     "md5": md5s}
    json.dump(out, open(os.path.join(ROOT, "tests", "golden", "h265.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
