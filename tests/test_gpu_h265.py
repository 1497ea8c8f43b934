"""H.265 pictures (intra, and P / B with motion compensation) reconstructed on gfx950 (m2dec_amd/csrc/hip/h265_hip.hip) through h265d_func, bit-exact
against the goldens the CPU oracle produced (tests/golden/h265.json, tests/test_h265_cpu.py).  Parity
against the reference itself is unpinned (no reference-produced H.265 output exists here)."""
import json
import os

import pytest

import m2dec_amd
from test_h265_cpu import h265_stream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "h265.json")))


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLD))
def test_hip_h265_matches_golden(built, name):
    data = h265_stream(name)
    md5s, err = m2dec_amd.decode_h265(data, device=0)
    assert err == -2
    assert md5s == GOLD[name]["md5"]


PB = sorted(GOLD)  # (the intra streams take the row kernel either way)


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"M2DEC_AMD_H265_CTU_GRID": "0"}, {"M2DEC_AMD_H265_STREAMS": "1"},
                                 {"M2DEC_AMD_H265_STREAMS": "8"}, {"M2DEC_AMD_H265_WAVES": "2"},
                                 {"M2DEC_AMD_H265_WAVES": "2", "M2DEC_AMD_H265_CTU_GRID": "0"}],
                         ids=["rows", "one_stream", "eight_streams", "one_wave_per_plane", "one_wave_rows"])
def test_hip_h265_inter_variants(built, monkeypatch, env):
    """P / B pictures through the row kernel (the CTU-grid kernel's predecessor), on one stream (every
    dependency in stream order), on 8 streams (every one an event wait), and with one wave per plane in the
    CTU kernels instead of two (no intra-CTU block scheduler): each bit-exact."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for name in PB:
        md5s, err = m2dec_amd.decode_h265(h265_stream(name), device=0)
        assert err == -2
        assert md5s == GOLD[name]["md5"], name


@pytest.mark.gpu
def test_mfma_idct_probe(built):
    """The 16 x 16 / 32 x 32 inverse DCT on the int8 matrix cores (m2dec_amd/csrc/hip/h265_mfma.h, the CTU kernels'
    path) equals the reference's two-pass integer transform on 1000 random blocks per size, int16 extremes
    included (tools/mfma_idct_probe.hip; the decomposition itself: tests/test_h265_mfma_cpu.py)."""
    import subprocess
    probe = os.path.join(ROOT, "tools", "_build", "mfma_idct_probe")
    r = subprocess.run([probe, "1000"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "N=16: 0 of 1000 blocks differ" in r.stdout and "N=32: 0 of 1000 blocks differ" in r.stdout
