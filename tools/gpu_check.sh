#!/bin/bash
# GPU parity run: pytest -m gpu; on failure, per-picture HIP-vs-oracle diffs of every synthetic stream.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
if [ $rc -ne 0 ]; then
  python - > gpurun_out/gen_streams.log 2>&1 <<'PY'
import sys; sys.path.insert(0, '.')
from tests._streams import GOLDEN, stream
for n in GOLDEN:
    open(f'/tmp/{n}.264', 'wb').write(stream(n))
PY
  for n in $(python -c "import json;print(' '.join(json.load(open('tests/golden/synthetic.json'))))"); do
    timeout -k 10 300 python -m tests.diag_dual /tmp/$n.264 > gpurun_out/diag_$n.log 2>&1
    r=$?
    echo "diag $n rc=$r"
    if [ $r -ge 124 ] || [ $r -eq 134 ] || [ $r -eq 139 ]; then exit $r; fi
  done
fi
exit 0
