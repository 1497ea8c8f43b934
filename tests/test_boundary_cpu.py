"""The caller-ownership contract of the reference API, driven exactly as the
reference's application layer drives h264d_func (tests/harness/m2decoder_like.cpp mirrors
src/app/m2decoder.h + frames.h): the context is plain `new[]` memory freed with `delete[]` and never
released, and the header callback deletes the frames and allocates new ones when they are not
sufficient (m2decoder.h:39-80).  CPU: the oracle reconstructs (test-only checker); the GPU twin is
tests/test_gpu_boundary.py.

Streams: F1 (the reference-pinned fixture, 320x240, 1 reference frame) concatenated with generator
streams that (a) fit F1's frames (no reallocation), (b) need more frames of the same size, (c) change
the picture size.  When the callback reallocates, frames still waiting in the DPB point at the new,
unwritten memory (in the reference too), so only the frames handed out before the reallocation and the
second stream's frames are defined; both must be exact."""
import os
import subprocess

import pytest

from tests._oracle import ORACLE_PATH, golden_md5s

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tools", "_build", "m2decoder_like")
GEN = os.path.join(ROOT, "tools", "_build", "h264gen")
F1 = os.path.join(ROOT, "tests", "golden", "f1_realshort.264")

# (name, generator arguments): a fits F1's 18 frames, b needs 20 of the same size, c is 352x288
SECOND = {
    "fit": ["--preset", "cov_cabac", "--seed", "11", "--frames", "10", "--size", "320x240",
            "--set", "num_ref_frames=1", "--set", "l0_active=1", "--set", "l1_active=1"],
    "more": ["--preset", "cov_cabac", "--seed", "12", "--frames", "10", "--size", "320x240"],
    "resize": ["--preset", "cov_cabac", "--seed", "13", "--frames", "10", "--size", "352x288"],
}


def gen(tmp_path, name):
    out = str(tmp_path / f"{name}.264")
    subprocess.run([GEN, *SECOND[name], "-o", out], check=True, stderr=subprocess.DEVNULL)
    return out


def harness(args, oracle=True, env=None, timeout=240):
    cmd = [HARNESS] + (["-o", ORACLE_PATH] if oracle else []) + args
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run(cmd, capture_output=True, timeout=timeout, env=e)
    assert r.returncode == 0, (r.returncode, r.stderr.decode()[-2000:])
    lines = [ln.rstrip("\r") for ln in r.stdout.decode().split("\n") if ln]
    md5 = [ln for ln in lines if not ln.startswith("#")]
    return lines, md5


def iters(lines):
    out = []
    for ln in lines:
        if ln.startswith("#iter"):
            f = ln.split()
            out.append({f[k]: int(f[k + 1]) for k in range(2, len(f) - 1, 2)})
    return out


def check_concat(lines, f1, second):
    """frames before the header callback's reallocation (if any) and the second stream's are exact"""
    frames = [ln for ln in lines if not ln.startswith("#iter")]
    assert len([f for f in frames if not f.startswith("#")]) == len(f1) + len(second)
    if "#realloc" in frames:
        k = frames.index("#realloc")
        assert frames[:k] == f1[:k]
        frames = [f for f in frames if f != "#realloc"]
    else:
        assert frames[:len(f1)] == f1
    assert frames[-len(second):] == second


@pytest.mark.parametrize("name", ["fit", "more", "resize"])
@pytest.mark.parametrize("threads", [0, 4])
def test_stream_switch_like_m2decoder(built, tmp_path, name, threads):
    s = gen(tmp_path, name)
    _, alone = harness(["-t", str(threads), s])
    cat = str(tmp_path / "cat.264")
    with open(cat, "wb") as f:
        f.write(open(F1, "rb").read() + open(s, "rb").read())
    lines, _ = harness(["-t", str(threads), cat])
    f1 = golden_md5s(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"))
    check_concat(lines, f1, alone)
    if name == "fit":
        assert "#realloc" not in lines


def test_dropped_contexts_are_reclaimed(built, tmp_path):
    """20 decoders created and dropped (delete[] of the context, no release), half of them mid-stream:
    the thread count never grows (the parse pool is per process) and the states are reclaimed."""
    s = gen(tmp_path, "resize")
    f1 = golden_md5s(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"))
    # (the parse pool is sized for the host share, M2DEC_AMD_POOL_THREADS; 4 here to bound the count; the
    # copy crews, M2DEC_AMD_COPY_CREW, 2 x 3 threads, are process-wide too)
    lines, md5 = harness(["-t", "4", "-n", "10", "-m", "7", F1, s], env={"M2DEC_AMD_POOL_THREADS": "4"})
    st = iters(lines)
    assert len(st) == 10
    assert len({x["threads"] for x in st}) == 1 and st[0]["threads"] <= 1 + 4 + 6
    assert max(x["contexts"] for x in st) <= 2
    assert md5[:7] == f1[:7]
    lines, md5 = harness(["-t", "4", "-n", "10", F1])
    st = iters(lines)
    assert md5 == f1 * 10
    assert all(x["contexts"] == 1 for x in st)


def test_context_cap_without_address_reuse(built, tmp_path):
    """-k: contexts are never freed, so no address is reused and the library cannot tell a dropped
    context from an idle one: the registry stays at M2DEC_AMD_MAX_CONTEXTS by reclaiming the least
    recently used finished (or long idle) state, and RSS stops growing once it is there."""
    s = gen(tmp_path, "fit")
    lines, md5 = harness(["-t", "4", "-n", "14", "-k", F1, s], env={"M2DEC_AMD_MAX_CONTEXTS": "6"})
    st = iters(lines)
    assert max(x["contexts"] for x in st) <= 6
    assert st[-1]["evicted"] >= 2 * 14 - 6
    assert {x["threads"] for x in st} == {st[0]["threads"]}
    rss = [x["rss_kb"] for x in st]
    assert rss[-1] < rss[4] * 1.3 + 20000, rss
    # mid-stream drops are reclaimed only once idle for M2DEC_AMD_IDLE_EVICT_S
    lines, md5 = harness(["-t", "4", "-n", "8", "-k", "-m", "5", F1, s],
                         env={"M2DEC_AMD_MAX_CONTEXTS": "4", "M2DEC_AMD_IDLE_EVICT_S": "0"})
    st = iters(lines)
    assert max(x["contexts"] for x in st) <= 4


def test_abandoned_contexts_hit_the_hard_ceiling(built, tmp_path):
    """contexts dropped mid-stream without release and never freed (-k: no address reuse, so no
    reclaim on init) are not evictable under the cap unless idle eviction is opted into; the registry still
    stops at twice M2DEC_AMD_MAX_CONTEXTS by evicting the least recently used state idle for
    M2DEC_AMD_HARD_IDLE_S."""
    s = gen(tmp_path, "fit")
    env = {"M2DEC_AMD_MAX_CONTEXTS": "3", "M2DEC_AMD_HARD_IDLE_S": "0"}
    lines, md5 = harness(["-t", "4", "-n", "12", "-k", "-m", "5", F1, s], env=env)
    st = iters(lines)
    assert len(st) == 12
    assert max(x["contexts"] for x in st) <= 6
    assert st[-1]["evicted"] >= 12 * 2 - 6
    f1 = golden_md5s(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"))
    assert md5[:5] == f1[:5]
    # without the hard ceiling's idle time reached, nothing mid-stream is evicted: the registry grows
    lines, _ = harness(["-t", "4", "-n", "4", "-k", "-m", "5", F1, s],
                       env={"M2DEC_AMD_MAX_CONTEXTS": "3", "M2DEC_AMD_HARD_IDLE_S": "3600"})
    assert max(x["contexts"] for x in iters(lines)) == 8


def test_finished_undrained_contexts_are_kept(built, tmp_path):
    """after decode_picture returns -2, M2Decoder::decode still drains the DPB with
    `while (peek_decoded_frame(ctx, &frm, 1))` (m2decoder.h:136-141).  A state in that window must not be
    reclaimed when other contexts are created over the cap: four streams decoded to their end, none
    drained, at M2DEC_AMD_MAX_CONTEXTS=2 — all four stay, then every frame comes out exactly."""
    s = gen(tmp_path, "fit")
    _, plain = harness(["-t", "4", F1, s, F1, s])
    lines, md5 = harness(["-t", "4", "-p", "-k", F1, s, F1, s], env={"M2DEC_AMD_MAX_CONTEXTS": "2"})
    paused = [ln for ln in lines if ln.startswith("#paused")]
    assert paused and "contexts 4 evicted 0" in paused[0], paused
    assert md5 == plain
    # once drained they are reclaimable: the next contexts over the cap take their places
    lines, _ = harness(["-t", "4", "-n", "3", "-p", "-k", F1, s], env={"M2DEC_AMD_MAX_CONTEXTS": "2"})
    assert max(x["contexts"] for x in iters(lines)) <= 2
