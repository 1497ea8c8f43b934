cd $GRAFT_REPO_ROOT
export M2DEC_AMD_ASYNC_STATS=1
timeout -k 10 200 python -u - <<'PY' 2>&1 | tee gpurun_out/e2e_one.txt
import os, sys, time, ctypes
sys.path.insert(0, '.')
import m2dec_amd
from tests._streams import GOLDEN, stream
data = stream("c3_1080p_s1")
m2dec_amd.decode_stream_md5(data)
for dpb in (-1, 16):
    t0 = time.perf_counter(); got = m2dec_amd.decode_stream_md5(data, dpb=dpb); dt = time.perf_counter() - t0
    print("md5 path dpb", dpb, round(len(got)/dt, 1), "fps", got == GOLDEN["c3_1080p_s1"]["md5"], flush=True)
n = [0]
t0 = time.perf_counter()
m2dec_amd.decode_stream(data, md5=False, on_frame=lambda f: n.__setitem__(0, n[0] + 1))
print("no-md5 decode path", round(n[0]/(time.perf_counter()-t0), 1), "fps", flush=True)
PY
