import os, sys, time, ctypes
sys.path.insert(0, '/root/repo')
import m2dec_amd
from tests._streams import stream
data = stream("c3_1080p_s1")
for th in (0, 8):
    m2dec_amd.decode_stream(data, md5=False, parse_threads=th)
    t0 = time.perf_counter(); n = 0
    cnt = [0]
    def cb(f): cnt[0] += 1
    m2dec_amd.decode_stream(data, md5=False, on_frame=cb, parse_threads=th)
    dt = time.perf_counter() - t0
    print("decode no-md5 threads", th, round(cnt[0] / dt, 1), "fps", flush=True)
# md5 cost
import numpy as np
buf = np.zeros(1920*1088*3//2, np.uint8)
f = m2dec_amd.Frame(); f.luma = buf.ctypes.data; f.chroma = buf.ctypes.data + 1920*1088; f.width = 1920; f.height = 1088
f.crop[3] = 8
t0 = time.perf_counter()
for i in range(20): m2dec_amd.frame_md5(f)
print("md5 ms/frame", round((time.perf_counter() - t0) / 20 * 1e3, 2))
t0 = time.perf_counter()
tr = m2dec_amd.Trace(data)
print("parse-only (trace) fps", round(60 / (time.perf_counter() - t0), 1))
