"""MPEG-1/2 video, BASELINE.json configs[0] (C1: MPEG-2 MP@ML 720x480 I-frame-only .m2v on the CPU path),
and P / B frame pictures, through the reference-shaped m2d_func table (m2dec_amd/csrc/host/mpeg2_dec.c)
with the host reconstruction (the gfx950 one: tests/test_gpu_mpeg2.py).

Pinned by the reference itself:
  * every VLC table against the codewords of the reference's own tables (tests/golden/mpeg2_vlc.json,
    tools/gen_mpeg2_vlc_golden.py) — both directions: each reference codeword decodes to the same value
    and no other codeword is accepted;
  * the reference's unit-test vectors (tests/golden/mpeg2_kat.json): the DCT-VLC table of
    mpeg2.cpp:1743-1753 and the intra-DC table of m2dec.cpp:142-217 at every dc_scale and predictor.
Whole streams ("parity unpinned": no reference-produced output exists) against the pure-Python
restatement oracle/mpeg2_oracle.py (which decodes with the reference's tables) and the goldens
tests/golden/m2v.json made by tools/make_m2v_goldens.py from both; the C1 stream also through the
h264dec CLI (`h264dec -O c1.m2v`), which the driver's GPU pass runs too (test_gpu_cli.py)."""
import ctypes
import hashlib
import json
import os
import subprocess
import sys

import pytest

import m2dec_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "m2v.json")))
VLC = json.load(open(os.path.join(ROOT, "tests", "golden", "mpeg2_vlc.json")))
KAT = json.load(open(os.path.join(ROOT, "tests", "golden", "mpeg2_kat.json")))
GEN = os.path.join(ROOT, "tools", "_build", "m2vgen")
SCAN0 = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14,
         21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60,
         61, 54, 47, 55, 62, 63]


def m2v_stream(name):
    g = GOLD[name]
    out = f"/tmp/m2v_{name}_{os.getpid()}.m2v"
    subprocess.run([GEN, "--preset", g["preset"], "--seed", str(g["seed"]), "--frames", str(g["frames"]), "-o", out],
                   check=True)
    data = open(out, "rb").read()
    os.unlink(out)
    assert hashlib.sha256(data).hexdigest() == g["sha256"], f"m2vgen output drifted for {name}"
    return data


def _b32(bits):
    return int(bits.ljust(32, "0")[:32], 2)


def _bytes(bits):
    bits = bits.replace(" ", "")
    bits += "0" * (-len(bits) % 8 + 64)
    return bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8))


@pytest.mark.parametrize("table", [0, 1])
def test_dct_tables_match_reference(built, table):
    L = m2dec_amd.lib()
    ref = {c[0]: (c[1], c[2]) for c in VLC[f"dct{table}"]}
    r, lv = ctypes.c_int(), ctypes.c_int()
    for bits, (run, level) in ref.items():
        n = L.m2dec_amd_m2v_dct_code(table, _b32(bits), ctypes.byref(r), ctypes.byref(lv))
        exp = (-1, 3 if level else 0) if run < 0 else (run, level)
        assert (n, r.value, lv.value) == (len(bits), *exp), bits
    # no codeword the reference rejects: every 17-bit pattern decodes to a reference codeword or nothing
    for v in range(1 << 17):
        bits = format(v, "017b")
        n = L.m2dec_amd_m2v_dct_code(table, v << 15, ctypes.byref(r), ctypes.byref(lv))
        if n:
            assert bits[:n] in ref, bits[:n]
        else:
            assert not any(bits.startswith(c) for c in ref), bits


@pytest.mark.parametrize("table,key", [(0, "mb_inc_after0"), (1, "dc_luma"), (2, "dc_chroma"), (3, "motion_code")])
def test_vlc_tables_match_reference(built, table, key):
    L = m2dec_amd.lib()
    ref = {c[0]: c[1] for c in VLC[key]}
    v = ctypes.c_int()
    for bits, val in ref.items():
        assert (L.m2dec_amd_m2v_vlc_code(table, _b32(bits), ctypes.byref(v)), v.value) == (len(bits), val), bits
    for x in range(1 << 12):
        bits = format(x, "012b")
        n = L.m2dec_amd_m2v_vlc_code(table, x << 20, ctypes.byref(v))
        if n:
            assert bits[:n] in ref, bits[:n]
        else:
            assert not any(bits.startswith(c) for c in ref), bits


def test_reference_dct_vlc_kat(built):
    """mpeg2.cpp:1743-1798 test_parse_coef: MPEG-2 intra AC from scan index 1, flat-16 matrix, q_scale
    q_mapping[1][0] = 1; the coefficient at zigzag[pos] must equal `level`, `length` bits consumed."""
    L = m2dec_amd.lib()
    for k in KAT["dct_table0"]:
        coef = (ctypes.c_int16 * 64)()
        n = L.m2dec_amd_m2v_intra_ac(_bytes(k["input"]), 16, 1, 0, 0, 1, None, 0, coef)
        assert n == k["length"], k
        assert coef[SCAN0[k["pos"]]] == k["level"], k


def test_reference_intra_dc_kat(built):
    """m2dec.cpp:179-217 test_intra_dc: every vector at dc_scale 0..3 and predictor 0..254 returns
    clamp(ret + dc, 0, intra_dc_max) << dc_scale."""
    L = m2dec_amd.lib()
    v = ctypes.c_int()
    for k in KAT["intra_dc"]:
        data = _bytes(k["input"])
        for dc_scale in range(4):
            dc_max = (1 << (8 + 3 - dc_scale)) - 1
            for dc in range(255):
                assert L.m2dec_amd_m2v_intra_dc(data, 16, k["block_idx"], 3 - dc_scale, dc, ctypes.byref(v)) == \
                    len(k["input"])
                assert v.value == max(0, min(dc_max, k["ret"] + dc)) << dc_scale, (k, dc_scale, dc)


@pytest.mark.parametrize("name", ["cov_m2v_s1", "cov_m2v_s2", "cov_m2v_slices_s1", "cov_mpeg1_s1"])
def test_m2v_coverage_matches_oracle_and_golden(built, name):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import mpeg2_oracle
    data = m2v_stream(name)
    got = m2dec_amd.decode_m2v(data)
    assert got == GOLD[name]["md5"]
    assert got == mpeg2_oracle.decode(data)


def test_c1_matches_golden(built):
    got, err = m2dec_amd.decode_table_frames("m2d_func", m2v_stream("c1_480p_s1"))
    assert err == -1  # m2d_decode_data returns -1 at the end of the data (mpeg2.cpp:1583-1604)
    assert got == GOLD["c1_480p_s1"]["md5"]


def test_c1_cli_md5(built, tmp_path):
    """`h264dec -O c1.m2v` writes <basename>.out with one MD5 line per frame (filewrite.h:99-124); the exit
    status is the reference's: the last decode_picture result, -1 for MPEG-2's end of data."""
    src = tmp_path / "c1.m2v"
    src.write_bytes(m2v_stream("c1_480p_s1"))
    r = subprocess.run([os.path.join(ROOT, "m2dec_amd", "lib", "h264dec"), "-O", str(src)], cwd=tmp_path,
                       capture_output=True)
    assert r.returncode == 255, r.stderr
    out = (tmp_path / "c1.out").read_bytes()
    assert out == b"".join(m.encode() + b"\r\n" for m in GOLD["c1_480p_s1"]["md5"])
    r = subprocess.run([os.path.join(ROOT, "m2dec_amd", "lib", "h264dec"), "-x", "-e", "-O", str(src)], cwd=tmp_path,
                       capture_output=True)
    assert r.returncode == 0 and (tmp_path / "c1.out").read_bytes() == out


PB_SMALL = ["cov_m2v_pb_s1", "cov_m2v_pb_s2", "cov_m2v_pb_field_s1", "cov_m2v_pb_field_s2", "cov_mpeg1_pb_s1"]


@pytest.mark.parametrize("name", PB_SMALL)
def test_m2v_pb_matches_oracle_and_golden(built, name):
    """P / B frame pictures (every macroblock type, skips, frame / field / dual-prime MC, field DCT,
    f_codes 1-4, lost slices) on the host reconstruction: the golden, and the oracle's restatement of
    mpeg2.cpp + motioncomp.cpp; no output depends on reference UB (CLIP255C domain, reads outside the
    reference frame)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import mpeg2_oracle
    data = m2v_stream(name)
    got = m2dec_amd.decode_m2v(data)
    assert m2dec_amd.m2v_last_checks() == (0, 0)
    assert got == GOLD[name]["md5"]
    assert mpeg2_oracle.decode(data) == GOLD[name]["md5"]


def test_c1_pb_matches_golden(built):
    """C1's geometry (720x480) with P / B pictures; its golden was checked against the oracle on every
    frame when it was made (tools/make_m2v_goldens.py)."""
    got, err = m2dec_amd.decode_table_frames("m2d_func", m2v_stream("c1_pb_480p_s1"))
    assert err == -1
    assert got == GOLD["c1_pb_480p_s1"]["md5"]
    assert m2dec_amd.m2v_last_checks() == (0, 0)


def test_m2v_pb_emptify_same_frames(built):
    """h264dec -e (emptify the output queue after each picture) delivers the same frames in the same order."""
    data = m2v_stream("cov_m2v_pb_s1")
    assert m2dec_amd.decode_m2v(data, emptify=True) == GOLD["cov_m2v_pb_s1"]["md5"]


def test_d_pictures_are_reported(built):
    """D pictures (picture_coding_type 4) are not decoded: decode_picture returns -1 at their header."""
    data = bytearray(m2v_stream("cov_m2v_s1"))
    k = data.find(b"\x00\x00\x01\x00", 100)  # the second picture header
    data[k + 5] = (data[k + 5] & 0xc7) | (4 << 3)  # picture_coding_type = D
    got, err = m2dec_amd.decode_table_frames("m2d_func", bytes(data))
    assert err == -1 and len(got) < GOLD["cov_m2v_s1"]["frames"]


def test_gpu_reconstruction_has_no_host_fallback(built):
    """decode_m2v(device=n) on a device that does not exist (or with no GPU at all) is an error, never a
    silent host decode."""
    with pytest.raises(RuntimeError):
        m2dec_amd.decode_m2v(m2v_stream("cov_m2v_pb_s1"), device=64)


@pytest.mark.parametrize("name", ["c1_480p_s1", "cov_m2v_pb_s1"])
def test_md5_driver_matches_golden(built, name):
    """m2dec_amd_decode_m2v_md5 (MD5 lines from the helper threads, host reconstruction) equals the goldens."""
    assert m2dec_amd.decode_m2v_md5(m2v_stream(name)) == GOLD[name]["md5"]
