"""Reproduce the harness hang of tests/test_gpu_boundary.py::test_gpu_stream_switch_like_m2decoder[fit]:
this process decodes on the GPU first (as test_gpu_batch does in the pytest process), then runs the HIP
harness as a child: once with M2DEC_AMD_SHARE=0, then with the shared budget and M2DEC_AMD_DEBUG=1."""
import os
import subprocess
import sys
import tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402
from tests.test_boundary_cpu import F1, HARNESS, gen  # noqa: E402

assert m2dec_amd.decode_stream_md5(stream("cov_cabac_s1"), device=0) == GOLDEN["cov_cabac_s1"]["md5"]
print("parent decoded", flush=True)
d = tempfile.mkdtemp()


class P:
    def __init__(self, p):
        self.p = p

    def __truediv__(self, o):
        return P(os.path.join(self.p, o))

    def __str__(self):
        return self.p


s = gen(P(d), "fit")
cat = os.path.join(d, "cat.264")
open(cat, "wb").write(open(F1, "rb").read() + open(s, "rb").read())
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for tag, extra in (("noshare", {"M2DEC_AMD_SHARE": "0"}), ("share", {"M2DEC_AMD_DEBUG": "1"})):
    env = dict(os.environ, **extra)
    with open(os.path.join(out, f"diag_harness_{tag}.err"), "w") as ferr:
        try:
            r = subprocess.run([HARNESS, cat], env=env, stdout=subprocess.PIPE, stderr=ferr, timeout=40)
            print(tag, "rc", r.returncode, "lines", len(r.stdout.splitlines()), flush=True)
        except subprocess.TimeoutExpired:
            print(tag, "TIMEOUT", flush=True)
            sys.exit(3)
