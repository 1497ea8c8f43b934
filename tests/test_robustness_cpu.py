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

# multi-slice pictures whose damaged slice headers overlap or skip MBs: the sequential parse (after the
# slice-parallel one refused the tiling) decoded more MBs than the picture arena holds and overflowed its
# coefficient pool (heap corruption), or reached the last MB with MBs of the picture never coded and
# submitted their stale records (an out-of-range coefficient offset).  These seeds hit both before the
# fix (h264_slice_data: MB_ROOM, mbs_coded); each variant is decoded several times with 2 and 4 workers.
H264_SLICES = MUTATE + textwrap.dedent("""
    import sys
    sys.path.insert(0, ROOT)
    import m2dec_amd
    from tests._oracle import OracleBackend
    from tests._streams import stream
    done = 0
    data = stream("cov_slices_s1")
    for seed, idx in [(1000, 11), (1001, 7), (2000, 11), (2010, 4), (3000, 0), (3012, 4), (4002, 4)]:
        d = variants(data, seed, 12)[idx]
        for threads in (2, 4, 2, 4):
            with OracleBackend() as ob:
                try:
                    m2dec_amd.decode_stream(d, backend=ob.be, parse_threads=threads)
                except RuntimeError:
                    pass
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


def test_damaged_slices_overlapping(built):
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + H264_SLICES], capture_output=True, timeout=600,
                       cwd=ROOT)
    assert r.returncode == 0, (r.returncode, r.stderr.decode()[-3000:])
    assert b"decoded 28" in r.stdout, r.stdout.decode()[-500:]


H265_RPS_CHAIN = textwrap.dedent("""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, ROOT + "/tests")
    import m2dec_amd
    from _oracle import Oracle265Backend
    from test_h265_cpu import h265_stream

    class W:
        def __init__(self):
            self.bits = []
        def u(self, v, n):
            self.bits += [(v >> (n - 1 - i)) & 1 for i in range(n)]
        def ue(self, v):
            v += 1
            n = v.bit_length()
            self.u(0, n - 1)
            self.u(v, n)
        def rbsp(self):
            self.bits.append(1)
            while len(self.bits) % 8:
                self.bits.append(0)
            raw = bytes(int("".join(map(str, self.bits[i:i + 8])), 2) for i in range(0, len(self.bits), 8))
            out, z = bytearray(), 0
            for c in raw:  # emulation prevention
                if z >= 2 and c <= 3:
                    out.append(3)
                    z = 0
                out.append(c)
                z = z + 1 if c == 0 else 0
            return bytes(out)

    def sps(chain):
        w = W()
        w.u(0, 4); w.u(0, 3); w.u(1, 1)
        w.u(1, 8); w.u(0x60000000, 32); w.u(0, 24); w.u(0, 24); w.u(93, 8)  # profile_tier_level, 96 bits
        w.ue(0); w.ue(1); w.ue(64); w.ue(64); w.u(0, 1)   # sps 0, 4:2:0, 64x64, no cropping
        w.ue(0); w.ue(0); w.ue(4)                          # 8-bit, log2_max_poc_lsb 8
        w.u(1, 1); w.ue(4); w.ue(0); w.ue(0)               # sub-layer ordering
        w.ue(0); w.ue(1); w.ue(0); w.ue(3); w.ue(1); w.ue(1)   # CB 8..16, TB 4..32, depths
        w.u(0, 1); w.u(0, 1); w.u(0, 1); w.u(0, 1)         # no scaling lists / AMP / SAO / PCM
        w.ue(chain)
        w.ue(1); w.ue(0); w.ue(0); w.u(1, 1)               # set 0: one negative picture (-1), used
        for i in range(1, chain):                           # set i from set i-1: delta_rps -1, every entry kept
            w.u(1, 1); w.u(1, 1); w.ue(0)
            w.bits += [1] * (i + 1)                         # used_by_curr_pic_flag of the i + 1 candidates
        w.u(0, 1); w.u(0, 1); w.u(0, 1); w.u(0, 1); w.u(0, 1)  # no long-term, TMVP, smoothing, VUI, ext
        return b"\\x00\\x00\\x00\\x01\\x42\\x01" + w.rbsp()

    data = h265_stream("cov_h265_a_s1")
    at = data.find(b"\\x00\\x00\\x00\\x01\\x42\\x01")
    end = data.find(b"\\x00\\x00\\x01", at + 4)
    assert at >= 0 and end > at
    for chain in (15, 16, 17, 40, 64):
        # set k holds k + 1 entries, so set 16 would be predicted from 16 (> 16 after prediction)
        forged = data[:at] + sps(chain) + data[end - (1 if data[end - 1] == 0 else 0):]
        with Oracle265Backend() as o:
            md5s, err = m2dec_amd.decode_h265(forged, backend=o.be)
        assert err in (-1, -2), err
        print("chain", chain, "frames", len(md5s), "err", err)
    print("done")
""")


def test_h265_chained_inter_rps_is_bounded(built):
    """an SPS whose inter-RPS predictions chain (each set one entry longer than the one it is
    predicted from) must end in an error once a set would exceed the 16 entries of a reference picture set,
    not write past h265_st_rps_t.delta_poc (a stack overflow of parse_sps's SPS copy)."""
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + H265_RPS_CHAIN], capture_output=True, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, (r.returncode, r.stderr.decode()[-3000:])
    assert b"done" in r.stdout, r.stdout.decode()[-500:]
