"""FileWriterMd5 lines (reference filewrite.h:11-29, 99-105): the cropped NV12 rows of a frame, luma then
chroma, through RFC 1321 MD5 — the scalar path, the stitched 2-3 frame path and the 16-lane multi-buffer path
(m2dec_amd_frames_md5, m2dec_amd/csrc/host/md5.c) against Python's hashlib on the same bytes."""
import ctypes
import hashlib

import numpy as np
import pytest

import m2dec_amd
from m2dec_amd import Frame


def make_frames(rng, n, w, h, crop, one_buffer=True):
    """n frames of w x h NV12 (random bytes) in one buffer (like the MD5 ring) or separate ones."""
    size = w * h * 3 // 2
    mem = [rng.integers(0, 256, size * n, dtype=np.uint8)] if one_buffer else \
        [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(n)]
    frames = (Frame * n)()
    for i in range(n):
        base = mem[0].ctypes.data + i * size if one_buffer else mem[i].ctypes.data
        frames[i].luma, frames[i].chroma = base, base + w * h
        frames[i].width, frames[i].height = w, h
        for k in range(4):
            frames[i].crop[k] = crop[k]
    return mem, frames


def expected(f):
    w, h = f.width, f.height
    l, r, t, b = f.crop
    luma = np.ctypeslib.as_array((ctypes.c_uint8 * (w * h)).from_address(f.luma)).reshape(h, w)
    chroma = np.ctypeslib.as_array((ctypes.c_uint8 * (w * h // 2)).from_address(f.chroma)).reshape(h // 2, w)
    data = luma[t:h - b, l:w - r].tobytes() + chroma[t // 2:(h - b) // 2, l:w - r].tobytes()
    return hashlib.md5(data).hexdigest()


def lines(frames, n):
    L = m2dec_amd.lib()
    out = ctypes.create_string_buffer(35 * n)
    assert L.m2dec_amd_frames_md5(frames, n, out) == 0
    return [out.raw[35 * i:35 * i + 32].decode() for i in range(n)]


@pytest.mark.parametrize("w,h,crop", [(1920, 1088, (0, 0, 0, 8)), (1280, 720, (0, 0, 0, 0)), (176, 144, (0, 0, 2, 6)),
                                      (48, 32, (0, 0, 0, 0)), (208, 120, (4, 6, 2, 2)), (16, 16, (0, 0, 0, 2))])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 16])
def test_frames_md5_matches_hashlib(built, w, h, crop, n):
    rng = np.random.default_rng(w * 31 + n)
    _mem, frames = make_frames(rng, n, w, h, crop)
    want = [expected(frames[i]) for i in range(n)]
    assert lines(frames, n) == want
    assert [m2dec_amd.frame_md5(frames[i]) for i in range(n)] == want


def test_frames_md5_separate_buffers(built):
    rng = np.random.default_rng(5)
    _mem, frames = make_frames(rng, 16, 320, 240, (0, 0, 0, 0), one_buffer=False)
    want = [expected(frames[i]) for i in range(16)]
    assert lines(frames, 16) == want
    assert m2dec_amd.lib().m2dec_amd_frames_md5(frames, 17, ctypes.create_string_buffer(35 * 17)) == -1
