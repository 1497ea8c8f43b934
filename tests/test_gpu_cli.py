"""test.sh equivalent: `h264dec -O stream.264` writes stream.out; compare with the golden MD5s."""
import os
import subprocess

import pytest

from tests._oracle import ROOT
from tests._streams import GOLDEN, stream

APP = os.path.join(ROOT, "m2dec_amd", "lib", "h264dec")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["f1_realshort", "cov_cabac_s1", "cov_cavlc_s1", "c2_720p_s1"])
def test_cli_md5_matches_golden(built, tmp_path, name):
    if name == "f1_realshort":
        src = os.path.join(ROOT, "tests", "golden", "f1_realshort.264")
        want = open(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"), "rb").read()
    else:
        src = str(tmp_path / f"{name}.264")
        open(src, "wb").write(stream(name))
        want = "".join(m + "\r\n" for m in GOLDEN[name]["md5"]).encode()
    subprocess.run([APP, "-O", src], cwd=tmp_path, check=True, timeout=300)
    got = open(tmp_path / f"{os.path.splitext(os.path.basename(src))[0]}.out", "rb").read()
    assert got == want


@pytest.mark.gpu
def test_cli_skip_to_idr(built, tmp_path):
    """`h264dec -f 33` (M2Decoder::skip_frames, m2decoder.h:96-131): F1's SPS / PPS are replayed, decoding
    starts at the IDR before frame 33 (frame 30), and the output equals the tail of the full decode."""
    src = os.path.join(ROOT, "tests", "golden", "f1_realshort.264")
    want = open(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"), "rb").read()
    r = subprocess.run([APP, "-f", "33", "-O", src], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Skip " in r.stderr
    got = open(tmp_path / "f1_realshort.out", "rb").read()
    assert 0 < len(got) < len(want) and len(got) % 34 == 0
    assert want.endswith(got)


@pytest.mark.gpu
def test_cli_mpeg2_c1(built, tmp_path):
    """BASELINE.json configs[0] in the GPU pass too: `h264dec -O c1.m2v` (MPEG-2 on the CPU path)."""
    from tests.test_mpeg2_cpu import GOLD, m2v_stream
    src = tmp_path / "c1.m2v"
    src.write_bytes(m2v_stream("c1_480p_s1"))
    r = subprocess.run([APP, "-O", str(src)], cwd=tmp_path, capture_output=True, timeout=300)
    assert r.returncode == 255, r.stderr  # MPEG-2 decode_picture ends with -1 (mpeg2.cpp:1583-1604)
    assert (tmp_path / "c1.out").read_bytes() == b"".join(m.encode() + b"\r\n" for m in GOLD["c1_480p_s1"]["md5"])


@pytest.mark.gpu
def test_cli_h265(built, tmp_path):
    """`h264dec -O x.265` (M2Decoder MODE_H265 chosen by the extension, h264dec.cpp:153-154): the 1080p H.265
    intra stream reconstructed on the GPU, its .out equal to the oracle's goldens."""
    from tests.test_h265_cpu import GOLD as G265, h265_stream
    src = tmp_path / "c_h265.265"
    src.write_bytes(h265_stream("c_h265_1080p_s1"))
    r = subprocess.run([APP, "-O", str(src)], cwd=tmp_path, capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "c_h265.out").read_bytes() == b"".join(m.encode() + b"\r\n" for m in G265["c_h265_1080p_s1"]["md5"])


@pytest.mark.gpu
def test_cli_concurrent_processes_like_test_sh(built, tmp_path):
    """test.sh:2 runs `ls *.264 | parallel src/app/h264dec -O` — one decoder PROCESS per core, all on GPU 0.
    The decode path's forward-progress invariant (admission of k_picture launches against the device's
    resident capacity) must hold across those processes: the budget is the device's shared segment
    (devshare.c), not a per-process one.  Six h264dec -O processes started together, run once; every .out
    must equal its golden."""
    names = ["f1_realshort", "cov_cabac_s1", "cov_tools_s1", "c2_720p_s1", "c3_1080p_s1", "c4_1080p_s2"]
    want = {}
    for name in names:
        if name == "f1_realshort":
            src = tmp_path / "f1_realshort.264"
            src.write_bytes(open(os.path.join(ROOT, "tests", "golden", "f1_realshort.264"), "rb").read())
            want[name] = open(os.path.join(ROOT, "tests", "golden", "f1_realshort.md5"), "rb").read()
        else:
            (tmp_path / f"{name}.264").write_bytes(stream(name))
            want[name] = "".join(m + "\r\n" for m in GOLDEN[name]["md5"]).encode()
    env = dict(os.environ, M2DEC_AMD_SHARE_REPORT="1")
    procs = [subprocess.Popen([APP, "-O", f"{n}.264"], cwd=tmp_path, env=env, stdout=subprocess.DEVNULL,
                              stderr=subprocess.PIPE, text=True) for n in names]
    errs = {}
    for n, p in zip(names, procs):
        _, errs[n] = p.communicate(timeout=300)
        assert p.returncode == 0, (n, errs[n][-2000:])
    seen = [ln for n in names for ln in errs[n].splitlines() if ln.startswith("m2dec_amd budget:")]
    print("\n".join(seen))
    assert seen and all(" shared 1," in ln for ln in seen), "a process decoded without the device's shared budget"
    for n in names:
        assert (tmp_path / f"{n}.out").read_bytes() == want[n], n
