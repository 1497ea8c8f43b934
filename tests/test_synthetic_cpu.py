"""Synthetic streams on the CPU: generator determinism, parser vs generator cross-check, and the
oracle's per-frame MD5s against the committed goldens (regression of parser + oracle)."""
import pytest

import m2dec_amd
from tests import gen_check
from tests._oracle import OracleBackend, domain_violations
from tests._streams import GOLDEN, stream

COV = [n for n in GOLDEN if n.startswith("cov_")]
# the C4 set (c3 preset, seeds 2..8) is the same generator path as c3_1080p_s1; its goldens are checked
# on the GPU (tests/test_gpu_streams.py) and by every bench rank, not re-decoded by the CPU oracle here
CPU_SET = sorted(n for n in GOLDEN if not n.startswith("c4_"))


@pytest.mark.parametrize("name", CPU_SET)
def test_oracle_matches_golden(built, name):
    data = stream(name)
    domain_violations(reset=True)
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream(data, backend=ob.be)
    assert got == GOLDEN[name]["md5"]
    # the golden must not depend on CLIP255C table-domain UB in the reference (Appendix A #2)
    assert domain_violations() == 0


@pytest.mark.parametrize("preset,seed", [("cov_cavlc", 1), ("cov_cavlc", 5), ("cov_cabac", 1), ("cov_cabac", 7),
                                         ("cov_cabac4x4", 3), ("cov_wp", 2), ("cov_slices", 4), ("cov_tools", 3),
                                         ("cov_tools_cavlc", 3)])
def test_parser_matches_generator(built, tmp_path, preset, seed):
    errs = gen_check.check(preset, seed=seed, tmpdir=str(tmp_path))
    assert not errs, "\n".join(errs)


def test_parser_matches_generator_1080p(built, tmp_path):
    errs = gen_check.check("c3", seed=11, extra=("frames=5",), tmpdir=str(tmp_path))
    assert not errs, "\n".join(errs)


@pytest.mark.parametrize("direct", [0, 1])
def test_b_direct_motion_matches_generator(built, tmp_path, direct):
    """B-picture motion, direct blocks included, against the generator's spec restatement of
    temporal (direct=0) and spatial (direct=1) direct prediction (8.4.1.2): every MB exact, and
    direct blocks and B vectors actually compared."""
    import numpy as np
    from tests.gen_check import DUMP_DT, RecordingBackend, compare, generate
    out = str(tmp_path / f"d{direct}.264")
    generate("cov_cabac", out, out + ".dump", seed=9, extra=(f"direct={direct}",))
    dump = np.fromfile(out + ".dump", dtype=DUMP_DT)
    with OracleBackend() as ob:
        rec = RecordingBackend(ob.be)
        m2dec_amd.decode_stream(open(out, "rb").read(), backend=rec.be)
    st = {"direct": 0, "mv": 0}
    errs = compare(rec.pics, dump, stats=st)
    assert not errs, "\n".join(errs)
    assert int((dump["exact_mv"] == 0).sum()) == 0
    assert st["direct"] > 1000 and st["mv"] > 5000, st


def test_sps_scaling_lists_are_ignored(built, tmp_path):
    """The reference parses SPS scaling lists (6 + 8 lists, h264.cpp:280-296) and discards them:
    dequantisation stays flat.  The same stream with and without lists
    must reconstruct identically."""
    outs = []
    for sc in (0, 1):
        out = str(tmp_path / f"sc{sc}.264")
        gen_check.generate("cov_tools", out, seed=4, extra=(f"scaling={sc}",))
        with OracleBackend() as ob:
            outs.append(m2dec_amd.decode_stream(open(out, "rb").read(), backend=ob.be))
    assert len(outs[0]) == 16 and outs[0] == outs[1]
