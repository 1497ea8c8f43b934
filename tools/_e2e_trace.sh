set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2e_trace -o run -- python tools/_e2e_trace.py > gpurun_out/e2e_trace.log 2>&1
find gpurun_out/e2e_trace -name "*.csv" | head
