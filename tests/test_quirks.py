"""The reference quirks the GPU kernels reproduce are executed, not just coded:
the oracle counts each quirk path it takes (oracle_quirk_hits, oracle/recon_oracle.c), and a golden
stream must reach it — so the GPU tests that check that stream bit-exactly prove the kernel path.

  A#1  SSE2 int16 saturation of explicit bi-weighting   cov_wp_quirks (weights up to 127, bright pairs)
  A#16 int8 store of weight 128, explicit               cov_wp_quirks (log2 denominator 7, default weights)
  A#16 int8 wrap of implicit weight 128                 record level: no generated GOP gives
                                                        DistScaleFactor 512, so a c3 B slice's implicit
                                                        table is set to the wrapped (-64, -128) pair
  A#17 DC-only SWAR add at |adj| 200..255               cov_wp_quirks (8x8 blocks with one DC level)
  A#3  8x8 dequant truncation below QP 12               cov_cabac (QP 10..40)
  A#13 UMV (reference reads outside the frame)          every motion stream
  A#5  I_PCM deblock QP                                 cov_cabac (PCM MBs)
"""
import ctypes

import numpy as np
import pytest

import m2dec_amd
from tests._oracle import OracleBackend, domain_violations, quirk_hits
from tests._streams import GOLDEN, stream
from tests.gen_check import SET_FRAMES, SUBMIT, Picture

EXPECT = {"cov_wp_quirks_s1": ("sat16", "w128_explicit", "swar_big", "umv"), "cov_cabac_s1": ("deq8_trunc", "pcm", "umv")}


@pytest.mark.parametrize("name", sorted(EXPECT))
def test_quirk_paths_are_executed(built, name):
    quirk_hits()
    domain_violations()
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream(stream(name), backend=ob.be)
    hits = quirk_hits()
    assert got == GOLDEN[name]["md5"]
    assert domain_violations() == 0
    for q in EXPECT[name]:
        assert hits[q] > 0, (name, q, hits)


SLICE_IW = 8 + 2 * 32 * 3 * 2  # offsetof(m2r_slice_t, iw): wp_mode, log2wd[2], pad[5], w, o
SLICE_SIZE = SLICE_IW + 32 * 32 * 2


def wrap_implicit_weights(trace):
    """Set the implicit (w0, w1) of every implicit B slice to the int8-wrapped pair of w1 = 128:
    w0 = 64 - 128 = -64, w1 = (int8)128 = -128 (h264.cpp:7001-7025, h264.h:219)."""
    n = 0
    for p in trace.pics:
        for s in range(p.n_slices):
            base = trace.records_ptr + p.off_slice + s * SLICE_SIZE
            if ctypes.c_uint8.from_address(base).value != 2:  # M2R_WP_IMPLICIT
                continue
            for r0 in range(2):
                ctypes.memmove(base + SLICE_IW + (r0 * 32 + 0) * 2, bytes([0xc0, 0x80]), 2)
            n += 1
    return n


def oracle_decode_order(trace):
    """The CPU oracle over a trace's (possibly edited) records: one MD5 line per picture, decode order."""
    W, H = trace.width, trace.height
    crop = (ctypes.c_int * 4)()
    m2dec_amd.lib().m2dec_amd_trace_crop(trace.h, crop)
    out = []
    with OracleBackend() as ob:
        mem = [np.zeros(W * H * 3 // 2, np.uint8) for _ in range(trace.nslots)]
        frames = (m2dec_amd.Frame * trace.nslots)()
        for i, m in enumerate(mem):
            frames[i].luma = m.ctypes.data
            frames[i].chroma = m.ctypes.data + W * H
            frames[i].width, frames[i].height = W, H
            for k in range(4):
                frames[i].crop[k] = crop[k]
        SET_FRAMES(ob.be.set_frames)(ob.be.self, trace.nslots, frames, W, H)
        submit = SUBMIT(ob.be.submit)
        rec = trace.records_ptr
        for p in trace.pics:
            pic = Picture(p.width_mbs, p.height_mbs, p.slot, p.n_inter, p.n_coef, p.n_slices, p.n_intra, p.deblock,
                          rec + p.off_mb, rec + p.off_dbk, rec + p.off_slice, rec + p.off_inter, rec + p.off_coef,
                          p.n_slices, p.n_inter, p.n_coef, 0)
            assert submit(ob.be.self, ctypes.byref(pic)) == 0
            out.append(m2dec_amd.frame_md5(frames[p.slot]))
    return out


def test_implicit_wrap_reaches_the_oracle(built):
    tr = m2dec_amd.Trace(stream("cov_cabac_s1"))
    try:
        assert wrap_implicit_weights(tr) > 0
        quirk_hits()
        oracle_decode_order(tr)
        assert quirk_hits()["w128_implicit"] > 0
    finally:
        tr.close()


@pytest.mark.gpu
def test_implicit_wrap_hip_matches_oracle(built):
    """Record-level kernel parity for A#16's implicit case: the HIP batch replay of the edited records
    equals the oracle's reconstruction of the same records, picture by picture."""
    tr = m2dec_amd.Trace(stream("cov_cabac_s1"))
    try:
        assert wrap_implicit_weights(tr) > 0
        want = oracle_decode_order(tr)
        rp = m2dec_amd.HipReplay(tr, 0)
        try:
            got = rp.md5_decode_order()
        finally:
            rp.close()
    finally:
        tr.close()
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert len(got) == len(want) and not bad, f"pictures {bad[:10]} differ"
    assert len(set(want)) > 1
