#!/bin/bash
# Damaged-stream variants (tests/test_robustness_cpu.py's mutations, more of them) through the host parsers
# and the CPU oracles built with AddressSanitizer (host code only, no GPU).  Usage: bash tools/fuzz/run_asan.sh [N]
set -o pipefail
N=${1:-40}
R=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
gcc -O1 -g -fsanitize=address -fno-omit-frame-pointer -march=x86-64-v3 -std=gnu11 -I$R/include -I$R/m2dec_amd/csrc/host \
  -o $T/fuzz $R/tools/fuzz/fuzz_main.c $R/tools/fuzz/hip_stubs.c $R/m2dec_amd/csrc/host/*.c $R/oracle/recon_oracle.c \
  $R/oracle/h265_oracle.c -lpthread -lm || exit 1
python3 - "$T" "$N" <<'PY'
import os, sys, textwrap
R = os.getcwd()
sys.path.insert(0, R); sys.path.insert(0, R + "/tests")
src = open(R + "/tests/test_robustness_cpu.py").read()
ns = {}
exec(textwrap.dedent(src.split('MUTATE = textwrap.dedent("""')[1].split('""")')[0]), ns)
from tests._streams import stream
from test_h265_cpu import h265_stream
from test_mpeg2_cpu import m2v_stream
T, N = sys.argv[1], int(sys.argv[2])
sets = [("264", stream, ["cov_cabac_s1", "cov_cavlc_s1", "cov_slices_s1", "cov_tools_s1", "cov_wp_s1"]),
        ("265", h265_stream, ["cov_h265_a_s1", "cov_h265_b_s2", "cov_h265_c_s3", "cov_h265_hiqp_s1"]),
        ("m2v", m2v_stream, ["cov_m2v_s1", "cov_m2v_pb_s1", "cov_m2v_pb_field_s1"])]
for ext, get, names in sets:
    k = 0
    for name in names:
        for d in ns["variants"](get(name), 1000 + k, N):
            open(f"{T}/{ext}_{k}.bin", "wb").write(d)
            k += 1
PY
cd $R
for c in 264 265 m2v; do
  ASAN_OPTIONS=detect_leaks=0 $T/fuzz $c $T/${c}_*.bin > $T/$c.log 2>&1
  rc=$?; echo "$c: rc=$rc $(tail -1 $T/$c.log)"
  [ $rc -ne 0 ] && grep -E "ERROR|#[0-6] " $T/$c.log | head -12
done
rm -rf $T
