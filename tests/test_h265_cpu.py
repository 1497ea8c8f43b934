"""H.265 (h265d_func) on the CPU: the host parser against the generator's own syntax
dump, and the whole decode through M2Decoder with the CPU oracle's reconstruction (oracle/h265_oracle.c)
against the goldens tests/golden/h265.json (tools/make_h265_goldens.py).

Parity is "unpinned": the reference decoder is unbuildable here and holds no H.265
fixtures, so the goldens are the oracle's; the oracle restates h265.cpp's reconstruction with its quirks
(DC-only shortcut, luma tc QP clipped to 51, band offset without wrap, sign-hidden coefficient negated
after dequantisation) and the GPU path (tests/test_gpu_h265.py) must equal it bit for bit."""
import ctypes
import hashlib
import json
import os
import subprocess
import tempfile

import pytest

import m2dec_amd
from _oracle import Oracle265Backend, h265_violations

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "h265.json")))
GEN = os.path.join(ROOT, "tools", "_build", "h265gen")
SMALL = [k for k in GOLD if not k.startswith("c_")]


def h265_stream(name, dump=None):
    g = GOLD[name]
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "s.265")
        cmd = [GEN, "--preset", g["preset"], "--seed", str(g["seed"]), "--frames", str(g["frames"]), "-o", out]
        if dump:
            cmd += ["--dump", dump]
        subprocess.run(cmd, check=True)
        data = open(out, "rb").read()
    assert hashlib.sha256(data).hexdigest() == g["sha256"], f"h265gen output drifted for {name}"
    return data


def test_h265d_func_exported(built):
    L = m2dec_amd.lib()
    assert ctypes.c_void_p.in_dll(L, "h265d_func").value


@pytest.mark.parametrize("name", SMALL + ["c_h265_1080p_s1"])
def test_oracle_matches_golden(built, name):
    data = h265_stream(name)
    h265_violations(True)
    with Oracle265Backend() as o:
        md5s, err = m2dec_amd.decode_h265(data, backend=o.be)
    assert err == -2
    assert md5s == GOLD[name]["md5"]
    assert h265_violations(True) == 0


INTER = [k for k in GOLD if GOLD[k]["preset"] in ("cov_h265_p", "cov_h265_hb", "cov_h265_ldb", "cov_h265_pnodbk")]


@pytest.mark.parametrize("name", ["cov_h265_a_s1", "cov_h265_b_s2", "cov_h265_c_s3", "cov_h265_hiqp_s1"] + INTER)
def test_parser_matches_generator_syntax(built, name, tmp_path):
    """Every CU's luma / chroma modes and every residual level the parser reads equal what the generator
    wrote (tools/h265gen --dump), and each slice's CABAC data ends exactly on end_of_slice_segment_flag.
    P / B pictures add every coding unit's skip / part mode and every prediction block's merge index or AMVP
    direction with its final references and vectors: the parser's merge / AMVP / TMVP derivation
    (m2dec_amd/csrc/host/h265_dec.c) against the generator's own (tools/h265gen)."""
    gdump, ddump = str(tmp_path / "gen.txt"), str(tmp_path / "dec.txt")
    data = h265_stream(name, gdump)
    L = m2dec_amd.lib()
    L.m2dec_amd_h265_set_dump.argtypes = [ctypes.c_char_p]
    assert L.m2dec_amd_h265_set_dump(ddump.encode()) == 0
    try:
        with Oracle265Backend() as o:
            m2dec_amd.decode_h265(data, backend=o.be)
    finally:
        L.m2dec_amd_h265_set_dump(None)
    dec = open(ddump).read().splitlines()
    assert not [x for x in dec if x.startswith("error")]
    assert open(gdump).read().splitlines() == dec


def test_long_stream_follows_reference_dpb(built):
    """20 pictures over the reference's 8 frames and 16-entry DPB (h265.cpp:180-205, 4931-4976): output
    starts only once the DPB is full, the entry past the 16th is dropped, and frames are reused by the LRU
    — 18 frames out, as the golden records."""
    assert len(GOLD["cov_h265_a_long_s3"]["md5"]) == 18


HITS = ["merge_spatial", "merge_temporal", "merge_combined", "merge_zero", "no_bidir", "mvp_a", "mvp_b", "mvp_scaled",
        "mvp_temporal", "mvp_zero", "bi", "lowdelay", "not_lowdelay", "col_stale", "bs_motion", "intra_cu"]


def test_inter_goldens_cover_the_derivation(built):
    """The P / B goldens reach every branch of the inter derivation: merge candidates of each kind selected
    (spatial, temporal — B slices only: a P slice's temporal candidate leaves its L1 reference unset in the
    reference, h265.cpp:3655, so h265gen never selects it —, combined bi-predictive, zero), 8x4 / 4x8 bi
    candidates cut to L0, AMVP predictors from A, B, scaled (mvp2nd), temporal and zero fill, bi-prediction,
    low-delay and non-low-delay B slices (TMVP list choice), a collocated_ref_idx kept from an earlier slice,
    motion-based deblocking strengths and intra CUs inside inter pictures."""
    L = m2dec_amd.lib()
    L.m2dec_amd_h265_parser_hits.argtypes = [ctypes.POINTER(ctypes.c_long), ctypes.c_int, ctypes.c_int]
    h = (ctypes.c_long * 16)()
    L.m2dec_amd_h265_parser_hits(h, 16, 1)
    total = [0] * 16
    p_temporal = 0
    for name in INTER:
        with Oracle265Backend() as o:
            md5s, err = m2dec_amd.decode_h265(h265_stream(name), backend=o.be)
        assert err == -2 and md5s == GOLD[name]["md5"]
        L.m2dec_amd_h265_parser_hits(h, 16, 1)
        total = [a + b for a, b in zip(total, h)]
        if GOLD[name]["preset"] in ("cov_h265_p", "cov_h265_pnodbk"):
            p_temporal += h[1]
    missing = [n for n, v in zip(HITS, total) if v == 0]
    assert not missing, missing
    assert p_temporal == 0


def test_truncated_p_slice_is_an_error(built):
    """A P slice whose header runs out of data: decode_picture returns -2 (the reference's error return,
    h265.cpp:4904-4906) and the pictures before it are still output."""
    data = bytearray(h265_stream("cov_h265_a_s1"))
    # the second picture's NAL: TRAIL_R (type 1); flip its slice_type ue(2) -> ue(0) is not a byte edit, so
    # instead cut the stream after the first picture and append a forged P-slice header
    first = data.find(b"\x00\x00\x00\x01\x02\x01")  # TRAIL_R start code + header
    assert first > 0
    forged = bytes(data[:first]) + b"\x00\x00\x00\x01\x02\x01" + bytes([0b11010000, 0x80, 0xC0, 0, 0, 0])  # first_slice 1, pps 0, slice_type ue 1 (P)
    with Oracle265Backend() as o:
        md5s, err = m2dec_amd.decode_h265(forged, backend=o.be)
    assert err == -2
    assert len(md5s) == 1


@pytest.mark.parametrize("name", ["cov_h265_a_long_s3", "c_h265_1080p_s1"])
def test_md5_driver_matches_golden(built, name):
    """m2dec_amd_decode_h265_md5: the MD5 lines hashed on the helper threads from the driver's copies equal
    the per-frame MD5s of the plain loop (and the goldens)."""
    data = h265_stream(name)
    with Oracle265Backend() as o:
        md5s, err = m2dec_amd.decode_h265_md5(data, backend=o.be)
    assert err == -2
    assert md5s == GOLD[name]["md5"]


@pytest.mark.parametrize("rps", [1, 2, 3])
def test_few_rps_sets_intra_stream(built, rps, tmp_path):
    """an all-intra stream whose SPS carries fewer than 8 short-term RPS sets.  The reference sizes its
    motion-field buffers by min(num_long_term_ref_pics_sps + num_short_term_ref_pic_sets, 8) (h265.cpp:121-128)
    and writes the current frame's for every picture, so a frame index at or above that count is reference UB
    (parity unpinned); the decoder keeps a motion field for every frame and decodes the stream to its end.  The
    application allocates that many frames too (get_info's frame_num), so the frame LRU and the output differ
    from the 8-set stream's, but every frame handed out holds one of the same pictures (cov_h265_a_long_s3: 20
    intra pictures)."""
    g = GOLD["cov_h265_a_long_s3"]
    out = str(tmp_path / "s.265")
    subprocess.run([GEN, "--preset", g["preset"], "--seed", str(g["seed"]), "--frames", str(g["frames"]), "--rps",
                    str(rps), "-o", out], check=True)
    data = open(out, "rb").read()
    assert hashlib.sha256(data).hexdigest() != g["sha256"]  # (a different SPS)
    with Oracle265Backend() as o:
        md5s, err = m2dec_amd.decode_h265(data, backend=o.be)
    assert err == -2
    assert md5s and set(md5s) <= set(g["md5"]), md5s


def test_worker_parse_error_matches_sequential(built, monkeypatch):
    """a slice-data error found by a parse-ahead worker.  The sequential path (and the reference,
    h265.cpp:4904) returns -2 at the failing picture and never outputs it or anything after it; with 8 workers
    decode_picture has already returned for later pictures, so the pipe rolls the DPB back to its state before
    the failed picture (less what was output meanwhile) and submits nothing after it.  Single-bit corruptions of
    the slice data that make the sequential parse fail: both paths give the same MD5 list and the same -2."""
    import random
    data = bytes(h265_stream("cov_h265_a_long_s3"))
    sc = b"\x00\x00\x00\x01"
    pos, i = [], data.find(sc)
    while i >= 0:
        pos.append(i)
        i = data.find(sc, i + 4)
    nals = [(p, (data[p + 4] >> 1) & 63) for p in pos]
    slices = [k for k, (_, t) in enumerate(nals) if t in (0, 1, 19)]
    with Oracle265Backend() as o:
        full, _ = m2dec_amd.decode_h265(data, backend=o.be)
    rng = random.Random(1)
    found = 0
    for _ in range(200):
        k = slices[rng.randrange(1, len(slices))]
        a, b = nals[k][0], nals[k + 1][0] if k + 1 < len(nals) else len(data)
        off = rng.randrange(a + 12, b - 2)
        bad = data[:off] + bytes([data[off] ^ (1 << rng.randrange(8))]) + data[off + 1:]
        monkeypatch.setenv("M2DEC_AMD_H265_THREADS", "0")
        with Oracle265Backend() as o:
            m0, e0 = m2dec_amd.decode_h265(bad, backend=o.be)
        if len(m0) >= len(full):
            continue  # (this corruption decodes to the end)
        monkeypatch.setenv("M2DEC_AMD_H265_THREADS", "8")
        with Oracle265Backend() as o:
            m8, e8 = m2dec_amd.decode_h265(bad, backend=o.be)
        assert (m8, e8) == (m0, e0) and e0 == -2
        found += 1
        if found == 6:
            break
    assert found == 6
