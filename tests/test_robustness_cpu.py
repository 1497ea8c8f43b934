"""Damaged streams through the three decoders' host parsers (H.264 `h264d_func`, H.265 `h265d_func`, MPEG-2
`m2d_func`), reconstruction by the CPU checkers: byte flips, zeroed runs, truncations and cut-and-spliced
NAL units must end in frames or an error return (-1 / -2, the reference's codes), never in a crash, a
hang or an out-of-bounds record.  Each codec runs in its own subprocess so that a crash is reported as a
test failure with its signal instead of ending the test session.  The oracles count record fields
outside what the reconstruction may address (oracle/recon_oracle.c, oracle/h265_oracle.c), and the GPU
back ends check the same bounds on the host before a launch (runtime.hip be_submit, h265_hip.hip
h_submit, m2v_hip.hip m2v_hip_submit), so a parser that let a damaged stream through with bad records
would show up here as an oracle fault.  Found this way (and fixed): MPEG-2 MBs parsed twice by overlapping
slices overflowing the picture's coefficient pool, address increments past the picture, records of an MB
abandoned mid-way keeping their coded-block pattern; an H.264 CAVLC run_before larger than the zeros left.
The same variants (and 200 more per codec) were run under AddressSanitizer with the host sources and both
oracles compiled in; the harness is in DESIGN.md §4."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MUTATE = textwrap.dedent("""
    import random

    def variants(data, seed, n):
        r = random.Random(seed)
        out = []
        for k in range(n):
            b = bytearray(data)
            kind = k % 4
            if kind == 0:    # scattered byte flips past the first parameter sets
                for _ in range(r.randint(1, 8)):
                    i = r.randrange(min(len(b) - 1, 40), len(b))
                    b[i] ^= 1 << r.randrange(8)
            elif kind == 1:  # a zeroed run (start codes and emulation prevention disturbed)
                i = r.randrange(40, len(b) - 64)
                b[i:i + r.randint(3, 64)] = bytes(r.randint(3, 64))[: len(b[i:i + 64])]
            elif kind == 2:  # truncated anywhere
                b = b[: r.randrange(16, len(b))]
            else:            # a slice of the stream spliced into another place
                i, j = sorted(r.randrange(40, len(b)) for _ in range(2))
                p = r.randrange(40, len(b))
                b = b[:p] + b[i:j] + b[p:]
            out.append(bytes(b))
        return out
""")

H264 = MUTATE + textwrap.dedent("""
    import sys
    sys.path.insert(0, ROOT)
    import m2dec_amd
    from tests._oracle import OracleBackend
    from tests._streams import stream
    done = 0
    for name in ["cov_cabac_s1", "cov_cavlc_s1", "cov_slices_s1"]:
        for d in variants(stream(name), hash(name) & 0xffff, 12):
            with OracleBackend() as ob:
                try:
                    m2dec_amd.decode_stream(d, backend=ob.be, parse_threads=2)
                except RuntimeError:
                    pass
            done += 1
    print("decoded", done)
""")

H265 = MUTATE + textwrap.dedent("""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, ROOT + "/tests")
    import m2dec_amd
    from _oracle import Oracle265Backend
    from test_h265_cpu import h265_stream
    done = 0
    for name in ["cov_h265_a_s1", "cov_h265_b_s2", "cov_h265_c_s3"]:
        for d in variants(h265_stream(name), hash(name) & 0xffff, 12):
            with Oracle265Backend() as o:
                md5s, err = m2dec_amd.decode_h265(d, backend=o.be)
            assert err in (-1, -2), err
            done += 1
    print("decoded", done)
""")

M2V = MUTATE + textwrap.dedent("""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, ROOT + "/tests")
    import m2dec_amd
    from test_mpeg2_cpu import m2v_stream
    done = 0
    for name in ["cov_m2v_s1", "cov_m2v_pb_s1", "cov_m2v_pb_field_s1"]:
        for d in variants(m2v_stream(name), hash(name) & 0xffff, 12):
            try:
                m2dec_amd.decode_m2v(d)
            except RuntimeError:
                pass
            done += 1
    print("decoded", done)
""")


@pytest.mark.parametrize("codec,script", [("h264", H264), ("h265", H265), ("m2v", M2V)], ids=["h264", "h265", "m2v"])
def test_damaged_streams_do_not_crash(built, codec, script):
    env = dict(os.environ, PYTHONHASHSEED="0")
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + script], capture_output=True, timeout=600,
                       env=env, cwd=ROOT)
    assert r.returncode == 0, (codec, r.returncode, r.stderr.decode()[-3000:])
    assert b"decoded 36" in r.stdout, r.stdout.decode()[-500:]
