"""The device-wide workgroup budget shared by every decoding process on one GPU (devshare.c; DESIGN §5
"Forward-progress invariant"; VERDICT r4 item 1: test.sh runs `parallel h264dec -O`, one decoder process per
core, on the same GPU).  No GPU: processes reserve and release units of a segment under a test key, as the
runtime does per k_picture launch, and the test checks that

  - the units held by all processes together never exceed the capacity (each holder adds its units to a
    counter shared by the test processes only after its reservation succeeded, and removes them before
    releasing, so counter <= the segment's total <= cap at every moment);
  - a holder killed while it holds units gives them back (its lease is reclaimed by the next reservation that
    does not fit);
  - the segment's file is gone once its last user closed it (nothing left in /dev/shm).
"""
import ctypes
import os
import signal
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "m2dec_amd", "lib", "libm2dec_amd.so")

WORKER = r"""
import ctypes, os, random, sys, time, mmap, struct
L = ctypes.CDLL(sys.argv[1])
L.m2dec_amd_share_open.restype = ctypes.c_void_p
L.m2dec_amd_share_open.argtypes = [ctypes.c_char_p, ctypes.c_int]
L.m2dec_amd_share_try.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.m2dec_amd_share_release.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.m2dec_amd_share_close.argtypes = [ctypes.c_void_p]
key, cap, mode = sys.argv[2], int(sys.argv[3]), sys.argv[4]
s = L.m2dec_amd_share_open(key.encode(), cap)
assert s, "open failed"
# the test's own shared counter: a file of 2 int64 (held units, max seen) updated under flock
import fcntl
cf = open(sys.argv[5], "r+b")
def add(d):
    fcntl.flock(cf, fcntl.LOCK_EX)
    cf.seek(0)
    held, mx = struct.unpack("qq", cf.read(16))
    held += d
    mx = max(mx, held)
    cf.seek(0)
    cf.write(struct.pack("qq", held, mx))
    cf.flush()
    fcntl.flock(cf, fcntl.LOCK_UN)
    return held
if mode == "churn":
    rnd = random.Random(os.getpid())
    mine = []
    got = 0
    t_end = time.time() + float(sys.argv[6])
    while time.time() < t_end:
        if mine and (rnd.random() < 0.5 or len(mine) > 6):
            u = mine.pop(rnd.randrange(len(mine)))
            assert add(-u) >= 0
            L.m2dec_amd_share_release(s, u)
        else:
            u = rnd.randint(1, cap // 3)
            if L.m2dec_amd_share_try(s, u):
                got += 1
                mine.append(u)
                assert add(u) <= cap, "units held by all processes exceed the capacity"
    for u in mine:
        add(-u)
        L.m2dec_amd_share_release(s, u)
    L.m2dec_amd_share_close(s)
    print("ok", got, flush=True)
elif mode == "hold":
    assert L.m2dec_amd_share_try(s, int(sys.argv[6]))
    print("holding", flush=True)
    time.sleep(600)
elif mode == "starve":  # a reservation that never fits, retried like SlotBudget::reserve for a while
    print("starving", flush=True)
    t_end = time.time() + float(sys.argv[6])
    while time.time() < t_end:
        assert not L.m2dec_amd_share_try(s, cap + 1)
        time.sleep(0.001)
    print("done", flush=True)
"""


def _lib():
    L = ctypes.CDLL(LIB)
    L.m2dec_amd_share_open.restype = ctypes.c_void_p
    L.m2dec_amd_share_open.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.m2dec_amd_share_try.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.m2dec_amd_share_release.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.m2dec_amd_share_state.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_int)] * 4 + \
        [ctypes.POINTER(ctypes.c_long)]
    L.m2dec_amd_share_close.argtypes = [ctypes.c_void_p]
    L.m2dec_amd_share_others_waiting.argtypes = [ctypes.c_void_p]
    return L


def _state(L, s):
    v = [ctypes.c_int() for _ in range(4)]
    r = ctypes.c_long()
    assert L.m2dec_amd_share_state(s, *[ctypes.byref(x) for x in v], ctypes.byref(r)) == 0
    return {"cap": v[0].value, "total": v[1].value, "mine": v[2].value, "procs": v[3].value, "reclaimed": r.value}


@pytest.fixture
def share_env(tmp_path, monkeypatch, built):
    monkeypatch.setenv("M2DEC_AMD_SHARE_DIR", str(tmp_path))
    return tmp_path


def test_four_processes_never_exceed_the_capacity(share_env):
    key, cap = f"test{os.getpid()}", 240
    counter = share_env / "counter"
    counter.write_bytes(b"\0" * 16)
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, "-c", WORKER, LIB, key, str(cap), "churn", str(counter), "3"],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for _ in range(4)]
    outs = [p.communicate(timeout=60) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
        assert o.startswith("ok"), o
        assert int(o.split()[1]) > 10, "a worker never got units: no real contention was tested"
    import struct
    held, mx = struct.unpack("qq", counter.read_bytes())
    assert held == 0
    assert 0 < mx <= cap
    assert mx > cap // 2, "the workers never held much of the budget together"
    # every process closed its handle: the segment's file is gone
    assert not [f for f in os.listdir(share_env) if f.startswith("m2dec_amd.budget.")]


def test_killed_holder_gives_its_units_back(share_env):
    L = _lib()
    key, cap = f"kill{os.getpid()}", 120
    counter = share_env / "counter"
    counter.write_bytes(b"\0" * 16)
    p = subprocess.Popen([sys.executable, "-c", WORKER, LIB, key, str(cap), "hold", str(counter), "100"],
                         stdout=subprocess.PIPE, text=True, start_new_session=True)
    try:
        assert p.stdout.readline().strip() == "holding"
        s = L.m2dec_amd_share_open(key.encode(), cap)
        assert s
        st = _state(L, s)
        assert st["total"] == 100 and st["procs"] == 1 and st["mine"] == 0
        assert not L.m2dec_amd_share_try(s, 30), "the live holder's units must not be handed out"
        assert L.m2dec_amd_share_try(s, 20)
        os.kill(p.pid, signal.SIGKILL)
        p.wait(timeout=30)
        # the next reservation that does not fit reclaims the dead process's lease
        assert L.m2dec_amd_share_try(s, 100)
        st = _state(L, s)
        assert st["total"] == 120 and st["mine"] == 120 and st["reclaimed"] == 100
        L.m2dec_amd_share_release(s, 120)
        assert _state(L, s)["total"] == 0
        L.m2dec_amd_share_close(s)
    finally:
        if p.poll() is None:
            os.kill(p.pid, signal.SIGKILL)
            p.wait(timeout=30)
    assert not [f for f in os.listdir(share_env) if f.startswith("m2dec_amd.budget.")]


def test_segment_outlives_one_user_while_another_holds_it(share_env):
    L = _lib()
    key = f"two{os.getpid()}"
    a = L.m2dec_amd_share_open(key.encode(), 60)
    b_env = dict(os.environ)
    # a second process opens the same segment and keeps units while this one closes
    (share_env / "c").write_bytes(b"\0" * 16)
    p = subprocess.Popen([sys.executable, "-c", WORKER, LIB, key, "60", "hold", str(share_env / "c"), "10"],
                         stdout=subprocess.PIPE, text=True, env=b_env, start_new_session=True)
    try:
        assert p.stdout.readline().strip() == "holding"
        L.m2dec_amd_share_close(a)
        files = [f for f in os.listdir(share_env) if f.startswith("m2dec_amd.budget.")]
        assert files, "the segment was removed while another process still uses it"
        c = L.m2dec_amd_share_open(key.encode(), 60)
        assert _state(L, c)["total"] == 10
        L.m2dec_amd_share_close(c)
    finally:
        os.kill(p.pid, signal.SIGKILL)
        p.wait(timeout=30)


def test_library_load_leaves_hw_queues_alone(built):
    """VERDICT r4 item 7 / ADVICE r4: loading the library must not configure the caller's HIP runtime."""
    # (the C environment, not os.environ: Python's copy is taken when the interpreter starts)
    code = ("import ctypes, sys; ctypes.CDLL(sys.argv[1]); g = ctypes.CDLL(None).getenv; "
            "g.restype = ctypes.c_char_p; print((g(b'GPU_MAX_HW_QUEUES') or b'unset').decode())")
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    r = subprocess.run([sys.executable, "-c", code, LIB], env=env, capture_output=True, text=True, check=True)
    assert r.stdout.strip() == "unset"
    # the explicit opt-in sets it, and a caller's own value wins
    code2 = ("import ctypes, sys; L = ctypes.CDLL(sys.argv[1]); g = ctypes.CDLL(None).getenv; "
             "g.restype = ctypes.c_char_p; print(L.m2dec_amd_configure_queues(8), g(b'GPU_MAX_HW_QUEUES').decode())")
    r = subprocess.run([sys.executable, "-c", code2, LIB], env=env, capture_output=True, text=True, check=True)
    assert r.stdout.split() == ["8", "8"]
    env["GPU_MAX_HW_QUEUES"] = "6"
    r = subprocess.run([sys.executable, "-c", code2, LIB], env=env, capture_output=True, text=True, check=True)
    assert r.stdout.split() == ["6", "6"]


def test_reaper_wakes_only_while_another_process_waits(share_env):
    """A process's budget reaper returns completed launches' units only while another process waits for units
    (its event queries otherwise contend with the decode threads' HIP calls); a waiter is seen while it retries
    and forgotten 100 ms after its last failed reservation."""
    L = _lib()
    key, cap = f"wait{os.getpid()}", 60
    s = L.m2dec_amd_share_open(key.encode(), cap)
    assert s
    try:
        assert L.m2dec_amd_share_others_waiting(s) == 0
        assert not L.m2dec_amd_share_try(s, cap + 1)  # this process's own failed reservation does not count
        assert L.m2dec_amd_share_others_waiting(s) == 0
        p = subprocess.Popen([sys.executable, "-c", WORKER, LIB, key, str(cap), "starve", "/dev/null", "1.0"],
                             stdout=subprocess.PIPE, text=True)
        assert p.stdout.readline().strip() == "starving"
        time.sleep(0.2)
        assert L.m2dec_amd_share_others_waiting(s) == 1
        assert p.stdout.readline().strip() == "done"
        p.wait(timeout=30)
        time.sleep(0.25)
        assert L.m2dec_amd_share_others_waiting(s) == 0
    finally:
        L.m2dec_amd_share_close(s)



# ---- round 6 hardening: owner-only segments, validated on open, liveness by lock

SEG_HEAD = 8  # magic, version (uint32 each), then the robust mutex (40 bytes on x86-64 glibc), cap, total


def _seg_file(share_env):
    files = [f for f in os.listdir(share_env) if f.startswith("m2dec_amd.budget.") and not f.endswith(".tmp")]
    assert len(files) == 1, files
    return share_env / files[0]


def _open2(L, key, cap):
    L.m2dec_amd_share_open2.restype = ctypes.c_void_p
    L.m2dec_amd_share_open2.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    why = ctypes.c_int(-1)
    s = L.m2dec_amd_share_open2(key.encode(), cap, ctypes.byref(why))
    return s, why.value


def _hold_in_child(share_env, key, cap, units):
    (share_env / "c").write_bytes(b"\0" * 16)
    p = subprocess.Popen([sys.executable, "-c", WORKER, LIB, key, str(cap), "hold", str(share_env / "c"), str(units)],
                         stdout=subprocess.PIPE, text=True, start_new_session=True)
    assert p.stdout.readline().strip() == "holding"
    return p


def test_segment_is_owner_only_and_named_per_user(share_env):
    L = _lib()
    s = L.m2dec_amd_share_open(f"mode{os.getpid()}".encode(), 60)
    assert s
    f = _seg_file(share_env)
    assert f.name.endswith(f".u{os.getuid()}")
    assert (f.stat().st_mode & 0o777) == 0o600
    L.m2dec_amd_share_close(s)


def test_group_mode_is_opt_in(share_env, monkeypatch):
    monkeypatch.setenv("M2DEC_AMD_SHARE_GROUP", "1")
    L = _lib()
    s = L.m2dec_amd_share_open(f"grp{os.getpid()}".encode(), 60)
    assert s
    f = _seg_file(share_env)
    assert f.name.endswith(f".g{os.getgid()}") and (f.stat().st_mode & 0o777) == 0o660
    L.m2dec_amd_share_close(s)


@pytest.mark.parametrize("damage", ["cap", "total", "lease_units", "version", "magic", "short"])
def test_corrupted_or_foreign_segment_is_refused_loudly(share_env, damage):
    """A segment file that is not a valid segment of this layout (another build's version, garbage in cap, total
    or a lease) is refused with a message, not silently replaced by a private budget; the back end then does not
    start (runtime.hip SlotBudget.refused)."""
    import struct
    L = _lib()
    key, cap = f"bad{damage}{os.getpid()}", 120
    p = _hold_in_child(share_env, key, cap, 30)  # a live user keeps the segment while the test damages it
    try:
        f = _seg_file(share_env)
        raw = bytearray(f.read_bytes())
        magic, version = struct.unpack_from("<II", raw, 0)
        cap_off = 8 + 40  # (after the pthread mutex)
        assert struct.unpack_from("<ii", raw, cap_off) == (cap, 30)
        lease0 = cap_off + 8 + 8  # cap, total, reclaimed (int64)
        if damage == "cap":
            struct.pack_into("<i", raw, cap_off, 10 ** 6)
        elif damage == "total":
            struct.pack_into("<i", raw, cap_off + 4, -5)
        elif damage == "lease_units":
            i = next(k for k in range(256) if struct.unpack_from("<i", raw, lease0 + 24 * k)[0] != 0)
            struct.pack_into("<i", raw, lease0 + 24 * i + 4, cap + 1)
        elif damage == "version":
            struct.pack_into("<I", raw, 4, version + 1)
        elif damage == "magic":
            struct.pack_into("<I", raw, 0, 0xdeadbeef)
        if damage == "short":
            f.write_bytes(bytes(raw[:100]))
        else:
            f.write_bytes(bytes(raw))
        r = subprocess.run([sys.executable, "-c",
                            "import ctypes, sys; L = ctypes.CDLL(sys.argv[1]); L.m2dec_amd_share_open2.restype = ctypes.c_void_p;"
                            "w = ctypes.c_int(-1); s = L.m2dec_amd_share_open2(sys.argv[2].encode(), int(sys.argv[3]), ctypes.byref(w));"
                            "print(bool(s), w.value)", LIB, key, str(cap)],
                           capture_output=True, text=True, timeout=60, env=dict(os.environ))
        assert r.stdout.split() == ["False", "2"], (r.stdout, r.stderr)
        assert "REFUSING the shared workgroup budget" in r.stderr
    finally:
        os.kill(p.pid, signal.SIGKILL)
        p.wait(timeout=30)


def test_dead_holder_found_by_its_lock_not_its_pid(share_env):
    """Liveness is the lease byte's open-file-description lock (dropped by the kernel at death, in any PID
    namespace): a lease whose pid names a live process but whose byte nobody locks is reclaimed."""
    import struct
    L = _lib()
    key, cap = f"lk{os.getpid()}", 120
    p = _hold_in_child(share_env, key, cap, 100)
    try:
        s = L.m2dec_amd_share_open(key.encode(), cap)
        assert not L.m2dec_amd_share_try(s, 30)  # the child's lock says it is alive
        # forge: the child's lease now names pid 1 (alive, not us) and the child dies: its lock goes
        f = _seg_file(share_env)
        os.kill(p.pid, signal.SIGKILL)
        p.wait(timeout=30)
        raw = bytearray(f.read_bytes())
        lease0 = 8 + 40 + 16
        i = next(k for k in range(256) if struct.unpack_from("<ii", raw, lease0 + 24 * k)[1] == 100)
        struct.pack_into("<i", raw, lease0 + 24 * i, 1)
        f.write_bytes(bytes(raw))
        assert L.m2dec_amd_share_try(s, 100), "a lease without its lock must be reclaimed even if its pid is alive"
        assert _state(L, s)["reclaimed"] == 100
        L.m2dec_amd_share_release(s, 100)
        L.m2dec_amd_share_close(s)
    finally:
        if p.poll() is None:
            os.kill(p.pid, signal.SIGKILL)
            p.wait(timeout=30)
