"""Latency of one m2dec_amd_frames_md5 batch of n 1080p frames (n = 1, 2, 3, 4, 8, 9, 16) on this host:
python3 tools/md5_batch_bench.py (M2DEC_AMD_MD5_STITCH=0: batches of 2-3 on the 16-lane kernel too)"""
import ctypes
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd
L = m2dec_amd.lib()
W, H = 1920, 1088
bufs = [(ctypes.create_string_buffer(os.urandom(W * H)), ctypes.create_string_buffer(os.urandom(W * H // 2))) for _ in range(16)]
F = (m2dec_amd.Frame * 16)()
for i, (y, c) in enumerate(bufs):
    F[i].width = W; F[i].height = H
    F[i].luma = ctypes.addressof(y); F[i].chroma = ctypes.addressof(c)
    F[i].crop[3] = 8
out = ctypes.create_string_buffer(35 * 16)
L.m2dec_amd_frames_md5.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
for n in (1, 2, 3, 4, 8, 9, 16):
    t = time.perf_counter(); reps = 5
    for _ in range(reps): L.m2dec_amd_frames_md5(F, n, out)
    print(n, "frames: %.2f ms per batch" % ((time.perf_counter() - t) / reps * 1e3))
