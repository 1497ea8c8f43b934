"""Synthetic streams through the product path (host parser -> HIP back end) on the GPU: every
frame's MD5 must equal the CPU oracle's golden."""
import os

import pytest

import m2dec_amd
from tests._streams import GOLDEN, stream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_hip_matches_golden(built, name):
    data = stream(name)
    got = m2dec_amd.decode_stream(data)
    want = GOLDEN[name]["md5"]
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert len(got) == len(want) and not bad, f"{name}: frames {bad[:10]} differ (of {len(want)})"


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_hip_batch_replay_matches_golden(built, name):
    """The bench path: every picture of the stream in ONE k_batch launch (slot reuse ordered on the
    device), each picture copied out before its slot is released; MD5s in output order."""
    data = stream(name)
    tr = m2dec_amd.Trace(data)
    rp = m2dec_amd.HipReplay(tr, 0)
    try:
        got = rp.md5_output_order()
    finally:
        rp.close()
        tr.close()
    want = GOLDEN[name]["md5"]
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert len(got) == len(want) and not bad, f"{name}: frames {bad[:10]} differ (of {len(want)})"


@pytest.mark.gpu
def test_hip_md5_driver_matches_golden(built):
    """m2dec_amd_decode_stream_md5: the same decode loop with the MD5s on a helper thread."""
    for name in ("cov_tools_s1", "c3_1080p_s1"):
        got = m2dec_amd.decode_stream_md5(stream(name))
        assert got == GOLDEN[name]["md5"], name


@pytest.mark.gpu
@pytest.mark.parametrize("env", [
    {"M2DEC_AMD_KCOPY": "0"},        # records up by SDMA copies instead of k_upload
    {"M2DEC_AMD_KCOPY_D2H": "1"},    # frames down by k_upload on a single decoder too
    {"M2DEC_AMD_KCOPY_D2H": "0"},    # frames down by SDMA with concurrent decoders too
    {"M2DEC_AMD_PRESTAGE": "0"},     # frames copied out at bind on the copy stream (round 5), not behind the kernel
], ids=["records_sdma", "frames_kernel", "frames_sdma", "copy_at_bind"])
def test_hip_copy_variants_match_golden(built, monkeypatch, env):
    """The upload / copy-out variants (read when a back end is created): one stream alone and two
    concurrent ones (several live back ends: the default copy-out is then k_upload), each bit-exact."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert m2dec_amd.decode_stream_md5(stream("c2_720p_s1")) == GOLDEN["c2_720p_s1"]["md5"]
    names = ["cov_tools_s1", "c3_1080p_s1"]
    got = m2dec_amd.decode_streams([stream(n) for n in names])
    for n, g in zip(names, got):
        assert g == GOLDEN[n]["md5"], n


@pytest.mark.gpu
def test_hip_concurrent_streams_match_golden(built):
    """Eight independent streams (the C4 set: c3 seeds 1..8) decoded at once on one GPU, one host
    thread and decoder context each (m2dec_amd_decode_streams_md5); every frame bit-exact."""
    names = ["c3_1080p_s1"] + [f"c4_1080p_s{s}" for s in range(2, 9)]
    got = m2dec_amd.decode_streams([stream(n) for n in names])
    for n, g in zip(names, got):
        want = GOLDEN[n]["md5"]
        bad = [i for i, (a, b) in enumerate(zip(g, want)) if a != b]
        assert len(g) == len(want) and not bad, f"{n}: frames {bad[:10]} differ (of {len(want)})"


@pytest.mark.gpu
@pytest.mark.parametrize("names", [
    # 320x192 coverage streams of different tools (CAVLC, CABAC, explicit weights, slices + cip + idc 2)
    ["cov_cabac_s1", "cov_cavlc_s1", "cov_wp_s1", "cov_tools_s1", "cov_cabac4x4_s1", "cov_wp_quirks_s1"],
    # the C4 set: eight 1080p streams in one replay (the gpu_recon_streams bench leg)
    ["c3_1080p_s1"] + [f"c4_1080p_s{s}" for s in range(2, 9)],
])
def test_hip_multistream_batch_replay_matches_golden(built, names):
    """Several independent streams in ONE replay (m2dec_amd_hip_replay_create_multi): pictures
    interleaved in one k_batch launch, each stream on its own frame slots; every frame of every
    stream bit-exact."""
    trs = [m2dec_amd.Trace(stream(n)) for n in names]
    rp = m2dec_amd.HipReplay(trs, 0)
    try:
        got = rp.md5_output_order()
    finally:
        rp.close()
        for t in trs:
            t.close()
    for n, g in zip(names, got):
        want = GOLDEN[n]["md5"]
        bad = [i for i, (a, b) in enumerate(zip(g, want)) if a != b]
        assert len(g) == len(want) and not bad, f"{n}: frames {bad[:10]} differ (of {len(want)})"


@pytest.mark.gpu
def test_forced_slow_waits_still_match_golden(built):
    """a hand-off wait past the report threshold (~1 s of polls by default; here every wait that
    polls at all, M2DEC_AMD_SPIN_REPORT=1) is reported once and waited on — every producer a wait points at holds
    a device-budget reservation, so waiting is the recovery — instead of ending the decode with an error as in
    round 5.  The stream still matches its golden, and the report reaches stderr.  (A separate process: the
    threshold is set when the process's first back end starts.)"""
    import subprocess
    import sys
    code = ("import m2dec_amd; from tests._streams import stream, GOLDEN; "
            "n = 'c3_1080p_s1'; print('OK' if m2dec_amd.decode_stream_md5(stream(n)) == GOLDEN[n]['md5'] else 'BAD')")
    env = dict(os.environ, M2DEC_AMD_SPIN_REPORT="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("OK"), r.stdout + r.stderr[-2000:]
    assert "waited past the report threshold" in r.stderr
