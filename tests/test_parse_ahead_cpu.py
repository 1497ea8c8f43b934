"""The parse-ahead pipeline (m2dec_amd/csrc/host/h264_async.c: slice data of several pictures parsed on
worker threads, marking / DPB / back-end calls on the caller's thread) through the CPU oracle back end:
every frame must equal the synchronous parser's golden, for single- and multi-slice, CAVLC and CABAC,
P and B (co-located store dependencies of direct prediction), deblocking idc 2 and constrained intra."""
import os

import pytest

import m2dec_amd
from tests._oracle import OracleBackend, golden_md5s
from tests._streams import GOLDEN, stream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["cov_cabac_s1", "cov_cabac_s2", "cov_cabac4x4_s1", "cov_cavlc_s1", "cov_wp_s1", "cov_slices_s1",
         "cov_tools_s1", "cov_tools_cavlc_s1", "c2_720p_s1"]


@pytest.mark.parametrize("threads", [1, 4])
@pytest.mark.parametrize("name", NAMES)
def test_parse_ahead_matches_golden(built, name, threads):
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream(stream(name), backend=ob.be, parse_threads=threads)
    assert got == GOLDEN[name]["md5"]


def test_parse_ahead_f1_matches_reference(built):
    data = open(os.path.join(ROOT, "tests", "golden", "f1_realshort.264"), "rb").read()
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream(data, backend=ob.be, parse_threads=3)
    assert got == golden_md5s(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"))


def test_parse_ahead_4k_multislice(built):
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream(stream("c5_4k_s1"), backend=ob.be, parse_threads=6)
    assert got == GOLDEN["c5_4k_s1"]["md5"]


@pytest.mark.parametrize("threads", [0, 4])
def test_skip_to_idr_cpu(built, threads):
    """h264dec -f (M2Decoder::skip_frames): the headers before the key frame are replayed, decoding
    starts at F1's IDR at frame 30 (the last key frame before frame 33), through the oracle back end;
    end of data inside one decode_picture call ends that call (the header replay's sentinel)."""
    data = open(os.path.join(ROOT, "tests", "golden", "f1_realshort.264"), "rb").read()
    gold = golden_md5s(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"))
    with OracleBackend() as ob:
        got, err = m2dec_amd.decode_table_frames("h264d_func", data, skip=33, backend=ob.be, parse_threads=threads)
    assert err == -2 and got == gold[30:]
    with OracleBackend() as ob:
        got, err = m2dec_amd.decode_table_frames("h264d_func", data, skip=20, backend=ob.be, parse_threads=threads)
    assert got == gold


@pytest.mark.parametrize("threads", [0, 4])
@pytest.mark.parametrize("dpb,emptify", [(-1, True), (16, False), (1, False)])
def test_output_calls_match_any_caller_pattern(built, threads, dpb, emptify):
    """The DPB options of h264dec (-d, -b, -e: M2Decoder::decode's emptify loop) change when frames are
    popped, never what they are: with the lookahead the API context still answers every peek / get
    exactly as the synchronous decoder."""
    name = "cov_cabac_s1"
    with OracleBackend() as ob:
        got, err = m2dec_amd.decode_table_frames("h264d_func", stream(name), dpb=dpb, emptify=emptify, backend=ob.be,
                                                 parse_threads=threads)
    with OracleBackend() as ob:
        ref, _ = m2dec_amd.decode_table_frames("h264d_func", stream(name), dpb=dpb, emptify=emptify, backend=ob.be,
                                               parse_threads=0)
    assert err == -2 and got == ref
    if dpb != 1:
        assert sorted(got) == sorted(GOLDEN[name]["md5"])


@pytest.mark.parametrize("name", ["c2_720p_s1", "cov_cabac_s1", "cov_slices_s1", "cov_tools_cavlc_s1"])
def test_decode_ahead(built, monkeypatch, name):
    """Back ends with bind (the oracle's, like the HIP one) get pictures as soon as they are parsed,
    named by virtual ids, from a submitter thread, before the API context reaches them (Stats.ahead
    counts those; M2DEC_AMD_AHEAD_ALL makes every picture go ahead, whatever the thread timing); the
    frames are the same with decode-ahead off (M2DEC_AMD_NO_AHEAD: submission in API order on the
    caller's thread, slots translated)."""
    monkeypatch.setenv("M2DEC_AMD_AHEAD_ALL", "1")
    st = m2dec_amd.Stats()
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream(stream(name), backend=ob.be, parse_threads=4, stats=st)
    assert got == GOLDEN[name]["md5"] and st.ahead == st.pictures
    monkeypatch.delenv("M2DEC_AMD_AHEAD_ALL")
    monkeypatch.setenv("M2DEC_AMD_NO_AHEAD", "1")
    st = m2dec_amd.Stats()
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream(stream(name), backend=ob.be, parse_threads=4, stats=st)
    assert got == GOLDEN[name]["md5"] and st.ahead == 0


@pytest.mark.parametrize("extra", [None, "0"])
@pytest.mark.parametrize("threads", [0, 4])
@pytest.mark.parametrize("name", ["c2_720p_s1", "cov_slices_s1"])
def test_md5_driver_holds_frames(built, monkeypatch, name, threads, extra):
    """The throughput driver (m2dec_amd_decode_stream_md5): frames hashed in place on helper threads,
    16 side by side, while the decoder keeps going — held frames are not reused until released
    (m2dec_hold_t), so the MD5 lines equal the goldens, in output order.  With no spare frames
    (M2DEC_AMD_MD5_EXTRA=0) the frame LRU has to wait for releases."""
    if extra is not None:  # and slow MD5 threads: frames stay held
        monkeypatch.setenv("M2DEC_AMD_MD5_EXTRA", extra)
        monkeypatch.setenv("M2DEC_AMD_MD5_DELAY_US", "1500000")
    st = m2dec_amd.Stats()
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream_md5_backend(stream(name), ob.be, parse_threads=threads,
                                                  md5_threads=1 if extra else 2, stats=st)
    assert got == GOLDEN[name]["md5"]
    if extra is not None and name == "c2_720p_s1":  # (cov_slices_s1 has fewer pictures than frames)
        assert st.hold_waits > 0


@pytest.mark.parametrize("name", ["cov_slices_s1", "cov_tools_s1", "cov_tools_cavlc_s1", "c5_4k_s1"])
def test_slice_parallel_parse(built, monkeypatch, name):
    """Multi-slice pictures parsed slice-parallel (several workers per picture, records packed in slice
    order, the MB-edge bS toward earlier slices computed after): every frame equals the golden, every
    multi-slice picture took that path (no sequential re-parse), and M2DEC_AMD_SLICE_PAR=0 (one worker
    per picture) gives the same frames."""
    want = GOLDEN[name]["md5"]
    with OracleBackend() as ob:
        st = m2dec_amd.Stats()
        got = m2dec_amd.decode_stream(stream(name), backend=ob.be, parse_threads=6, stats=st)
    assert got == want
    assert st.slice_par_pictures == len(want) and st.slice_par_fallbacks == 0, (st.slice_par_pictures,
                                                                                  st.slice_par_fallbacks)
    monkeypatch.setenv("M2DEC_AMD_SLICE_PAR", "0")
    with OracleBackend() as ob:
        st = m2dec_amd.Stats()
        assert m2dec_amd.decode_stream(stream(name), backend=ob.be, parse_threads=6, stats=st) == want
    assert st.slice_par_pictures == 0


_COL_CHILD = r"""
import sys
sys.path.insert(0, %r)
import m2dec_amd
from tests._oracle import OracleBackend
from tests._streams import GOLDEN, stream
with OracleBackend() as ob:
    got = m2dec_amd.decode_stream(stream(%r), backend=ob.be, parse_threads=6)
print('MD5OK', got == GOLDEN[%r]['md5'])
"""


@pytest.mark.parametrize("pipe", ["1", "0"])
@pytest.mark.parametrize("name", ["cov_cabac_s1", "cov_cabac_s2", "cov_wp_s1", "cov_reflists_s1"])
def test_col_row_pipelining(built, tmp_path, name, pipe):
    """Co-located row pipelining (h264_async.c deps_ready / job_run, h264_mb.c col_wait): a single-slice B
    picture starts while the anchor whose co-located store it reads is still being parsed, its direct
    prediction waiting per MB for the anchor's progress word.  The frames equal the goldens, and from the
    host timeline some B picture's parse starts before its anchor's ends (never with
    M2DEC_AMD_COL_PIPE=0)."""
    import csv
    import subprocess
    import sys
    tl = tmp_path / "tl.csv"
    # (anchors pause 2 ms per MB row, so that readers are picked while they run, whatever the host's CPUs)
    env = dict(os.environ, M2DEC_AMD_TIMELINE=str(tl), M2DEC_AMD_COL_PIPE=pipe, M2DEC_AMD_COL_PIPE_DELAY_US="2000")
    out = subprocess.run([sys.executable, "-c", _COL_CHILD % (ROOT, name, name)], env=env, capture_output=True,
                         text=True, timeout=600)
    assert "MD5OK True" in out.stdout, out.stdout + out.stderr[-2000:]
    start, end, typ = {}, {}, {}
    for r in csv.DictReader(open(tl)):
        if r["kind"] == "P":
            start[int(r["a"])], typ[int(r["a"])] = int(r["t_ns"]), int(r["b"])
        elif r["kind"] == "p":
            end[int(r["a"])] = int(r["t_ns"])
    early = 0
    for j in sorted(start):
        if typ[j] != 1:
            continue
        anchors = [k for k in start if k < j and typ[k] != 1]  # (its col writer: the last anchor before it)
        if anchors and start[j] < end[max(anchors)]:
            early += 1
    if pipe == "1":
        assert early > 0
    elif name != "cov_reflists_s1":  # (reordered lists: a B picture's anchor is not always the last one)
        assert early == 0


@pytest.mark.parametrize("name", ["cov_reflists_s1", "cov_reflists_s2", "cov_reflists_cavlc_s1", "cov_mmco5_s1",
                                  "cov_poc1_s1", "cov_tools_s1", "cov_wp_s1", "cov_slices_s1"])
def test_early_reference_submission(built, tmp_path, name):
    """Early submission (h264_async.c early_ok): a parsed reference picture goes to the back end ahead of
    older pictures still parsing, when every picture it may read is submitted and no older unsubmitted
    picture may read its buffer's previous content.  With the non-reference pictures held back
    (M2DEC_AMD_NONREF_DELAY_US, longer than the CPU checker's submission of a picture) the timeline shows early submissions ('S' events with b = 1) and the frames
    equal the goldens (list modification, MMCO 5, long-term references, POC types, weighted prediction,
    slices)."""
    import csv
    import subprocess
    import sys
    tl = tmp_path / "tl.csv"
    env = dict(os.environ, M2DEC_AMD_TIMELINE=str(tl), M2DEC_AMD_NONREF_DELAY_US="200000", M2DEC_AMD_EARLY="1")
    out = subprocess.run([sys.executable, "-c", _COL_CHILD % (ROOT, name, name)], env=env, capture_output=True,
                         text=True, timeout=600)
    assert "MD5OK True" in out.stdout, out.stdout + out.stderr[-2000:]
    early = sum(1 for r in csv.DictReader(open(tl)) if r["kind"] == "S" and r["b"] == "1")
    assert early > 0
