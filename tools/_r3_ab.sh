set -o pipefail
mkdir -p gpurun_out
./tools/_build/h264gen --preset c3 --seed 1 --frames 60 -o /tmp/c3.264 2>/dev/null
for i in 1 2 3 4 5 6; do echo "old $(LD_LIBRARY_PATH=tools/_build/ab ./tools/_build/pb /tmp/c3.264 1 | awk '{print $6}') new $(./tools/_build/pb /tmp/c3.264 1 | awk '{print $6}')"; done
