"""F1 (real-world High-profile CABAC stream) through the host parser + CPU oracle.

Pins the oracle: the 36 per-frame MD5s in tests/golden/f1_realshort.md5 are the reference
decoder's own `h264dec -O` output recorded in SURVEY.md §8c (whole-file md5 9df2923c...)."""
import hashlib
import os

from tests._oracle import OracleBackend, golden_md5s, ROOT

import m2dec_amd

GOLD = os.path.join(ROOT, "tests", "golden")


def test_f1_fixture_integrity():
    data = open(os.path.join(GOLD, "f1_realshort.264"), "rb").read()
    assert hashlib.sha256(data).hexdigest() == "ab39814a226782e5488b337e521bb02b261ea3d09e3fcf2fc21078b0a58ec9de"
    md5 = open(os.path.join(GOLD, "f1_realshort.md5"), "rb").read()
    assert hashlib.md5(md5).hexdigest() == "9df2923c50ef9ee23bd9acff7fa8a271"


def test_f1_oracle_matches_reference(built):
    data = open(os.path.join(GOLD, "f1_realshort.264"), "rb").read()
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream(data, backend=ob.be)
    assert got == golden_md5s(os.path.join(GOLD, "f1_realshort.md5"))
