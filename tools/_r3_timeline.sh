set -o pipefail
mkdir -p gpurun_out
python - > gpurun_out/timeline.log 2>&1 <<'PY'
import sys, os, time
sys.path.insert(0, '.')
import m2dec_amd
from tests._streams import stream, GOLDEN
d = stream('c3_1080p_s1')
for i in range(3):
    m2dec_amd.decode_stream_md5(d, device=0)
os.environ['M2DEC_AMD_ASYNC_STATS'] = '2'
st = m2dec_amd.Stats()
md5 = m2dec_amd.decode_stream_md5(d, device=0, stats=st)
print('ok', md5 == GOLDEN['c3_1080p_s1']['md5'], 'interval %.1f ms parse_cpu %.1f ms/frame' % (1e3*(st.t_end-st.t_start), 1e3*st.parse_cpu_s/60), flush=True)
PY
grep -v "^be_destroy\|^state_destroy" gpurun_out/timeline.log | tail -75
