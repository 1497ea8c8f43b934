#!/bin/bash
# Profile-guided build of the host library code: OUT/libm2dec_amd.so with the host objects compiled
# -fprofile-use from a training decode of streams that are NOT the bench's (c3 seed 11, c2 seed 9, c5 seed 9,
# 20 pictures each) through the null back end, parse on the caller's thread and on 4 workers.
# Usage: tools/pgo_build.sh OUT
set -e -o pipefail
OUT=${1:?out dir}
R=$(cd "$(dirname "$0")/.." && pwd)
W=$R/build/pgo
rm -rf "$W" && mkdir -p "$W/obj" "$W/lib" "$OUT"
CF="-O3 -g -fPIC -Wall -Wno-unused-parameter -std=gnu11 -I$R/include -I$R/m2dec_amd/csrc/host"
compile() { # $1 extra flags
  for f in "$R"/m2dec_amd/csrc/host/*.c; do
    b=$(basename "$f" .c); A="-march=x86-64-v3"; [ "$b" = cpucheck ] && A=""
    gcc $CF $A $1 -c "$f" -o "$W/obj/$b.o" &
  done
  wait
}
compile "-fprofile-generate -fprofile-update=atomic"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$W/lib/libm2dec_amd.so" "$W"/obj/*.o "$R"/build/hip/*.o -lpthread -lgcov
gcc -O2 -I"$R/include" -o "$W/train" "$R/tools/parse_bench.c" -L"$W/lib" -lm2dec_amd -Wl,-rpath,"$W/lib"
for s in "c3 11" "c2 9" "c5 9"; do
  set -- $s
  "$R/tools/_build/h264gen" --preset $1 --seed $2 --frames 20 -o "$W/t_$1.264" 2>/dev/null
  "$W/train" "$W/t_$1.264" 1 > /dev/null
done
compile "-fprofile-use -fprofile-partial-training -Wno-missing-profile"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libm2dec_amd.so" "$W"/obj/*.o "$R"/build/hip/*.o -lpthread
echo "pgo library: $OUT/libm2dec_amd.so"
