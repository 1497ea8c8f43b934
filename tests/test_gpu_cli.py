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
