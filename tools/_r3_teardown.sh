set -o pipefail
mkdir -p gpurun_out
python - > gpurun_out/teardown.log 2>&1 <<'PY'
import sys, os, time
sys.path.insert(0, '.')
os.environ['M2DEC_AMD_ASYNC_STATS'] = '1'
import m2dec_amd
from tests._streams import stream, GOLDEN
d = stream('c3_1080p_s1')
for i in range(4):
    st = m2dec_amd.Stats()
    t0 = time.perf_counter()
    md5 = m2dec_amd.decode_stream_md5(d, device=0, stats=st)
    t1 = time.perf_counter()
    print('step', i, 'ok', md5 == GOLDEN['c3_1080p_s1']['md5'], 'interval %.1f ms wall %.1f ms teardown %.1f ms setup %.1f ms' % (1e3*(st.t_end-st.t_start), 1e3*(t1-t0), 1e3*st.teardown_s, 1e3*st.setup_s), flush=True)
d5 = stream('c5_4k_s1')
for i in range(3):
    st = m2dec_amd.Stats()
    md5 = m2dec_amd.decode_stream_md5(d5, device=0, stats=st)
    print('c5 step', i, 'ok', md5 == GOLDEN['c5_4k_s1']['md5'], 'fps %.1f par %d fb %d teardown %.1f ms' % (16/(st.t_end-st.t_start), st.slice_par_pictures, st.slice_par_fallbacks, 1e3*st.teardown_s), flush=True)
PY
grep -v "^job" gpurun_out/teardown.log | grep -E "step|destroy|async:" | tail -40
