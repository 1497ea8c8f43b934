set -o pipefail
export M2DEC_AMD_LIB=build/dbg/libm2dec_amd_stampd.so
for n in 1 2; do M2DEC_AMD_REPLAY_LIMIT=$n M2DEC_AMD_REPLAY_ISOLATE_LAST=1 timeout -k 10 120 python tools/stamps_dbk.py > gpurun_out/stampd_$n.txt 2>&1 || exit $?; done
