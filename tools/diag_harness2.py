"""The harness hang with the shared budget (tools/diag_harness.py: every picture launched, then no exit): this
process decodes first, starts the HIP harness with the shared budget, and if it is still alive after 15 s
dumps its threads (/proc/<pid>/task/*: comm, wchan, syscall, stack of the user frames unavailable) and the
budget segment's leases, then kills it."""
import ctypes
import glob
import mmap
import os
import signal
import struct
import subprocess
import sys
import tempfile
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import m2dec_amd  # noqa: E402
from tests._streams import GOLDEN, stream  # noqa: E402
from tests.test_boundary_cpu import F1, HARNESS, SECOND, GEN  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
assert m2dec_amd.decode_stream_md5(stream("cov_cabac_s1"), device=0) == GOLDEN["cov_cabac_s1"]["md5"]
d = tempfile.mkdtemp()
s = os.path.join(d, "fit.264")
subprocess.run([GEN, *SECOND["fit"], "-o", s], check=True, stderr=subprocess.DEVNULL)
cat = os.path.join(d, "cat.264")
open(cat, "wb").write(open(F1, "rb").read() + open(s, "rb").read())
log = open(os.path.join(out, "diag2.txt"), "w")


def dump_proc(pid, tag):
    for t in sorted(glob.glob(f"/proc/{pid}/task/*")):
        def rd(n):
            try:
                return open(os.path.join(t, n)).read().strip()
            except OSError as e:
                return f"<{e.__class__.__name__}>"
        log.write(f"{tag} tid {os.path.basename(t)} comm {rd('comm')} wchan {rd('wchan')} syscall {rd('syscall')}\n")


def dump_seg():
    for f in glob.glob("/dev/shm/m2dec_amd.budget.*"):
        b = open(f, "rb").read()
        magic, ver = struct.unpack_from("II", b, 0)
        # pthread_mutex_t is 40 bytes at offset 8 (x86-64 glibc); its lock word first, owner tid at +8
        lockw, count, owner = struct.unpack_from("iIi", b, 8)
        cap, total, reclaimed = struct.unpack_from("iiq", b, 48)
        log.write(f"seg {f}: magic {magic:x} ver {ver} mutex lock {lockw:#x} owner {owner} cap {cap} total {total} reclaimed {reclaimed}\n")
        for i in range(256):
            pid, units, ctxs, pad, start = struct.unpack_from("iiiiQ", b, 64 + 24 * i)
            if pid:
                log.write(f"  lease {i}: pid {pid} units {units} contexts {ctxs} start {start}\n")


env = dict(os.environ, M2DEC_AMD_DEBUG="1")
p = subprocess.Popen([HARNESS, cat], env=env, stdout=subprocess.PIPE, stderr=open(os.path.join(out, "diag2_child.err"), "w"))
t0 = time.time()
while p.poll() is None and time.time() - t0 < 15:
    time.sleep(0.2)
if p.poll() is None:
    log.write(f"child {p.pid} alive after 15 s; parent {os.getpid()}\n")
    dump_proc(p.pid, "child")
    dump_proc(os.getpid(), "parent")
    dump_seg()
    log.flush()
    p.send_signal(signal.SIGKILL)
    p.wait()
    print("HUNG (dumped)", flush=True)
else:
    log.write(f"child exited rc {p.returncode}\n")
    print("exited", p.returncode, flush=True)
log.close()
