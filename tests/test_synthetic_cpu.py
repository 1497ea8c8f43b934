"""Synthetic streams on the CPU: generator determinism, parser vs generator cross-check, and the
oracle's per-frame MD5s against the committed goldens (regression of parser + oracle)."""
import pytest

import m2dec_amd
from tests import gen_check
from tests._oracle import OracleBackend
from tests._streams import GOLDEN, stream

COV = [n for n in GOLDEN if n.startswith("cov_")]
# the C4 set (c3 preset, seeds 2..8) is the same generator path as c3_1080p_s1; its goldens are checked
# on the GPU (tests/test_gpu_streams.py) and by every bench rank, not re-decoded by the CPU oracle here
CPU_SET = sorted(n for n in GOLDEN if not n.startswith("c4_"))


@pytest.mark.parametrize("name", CPU_SET)
def test_oracle_matches_golden(built, name):
    data = stream(name)
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream(data, backend=ob.be)
    assert got == GOLDEN[name]["md5"]


@pytest.mark.parametrize("preset,seed", [("cov_cavlc", 1), ("cov_cavlc", 5), ("cov_cabac", 1), ("cov_cabac", 7),
                                         ("cov_cabac4x4", 3), ("cov_wp", 2), ("cov_slices", 4)])
def test_parser_matches_generator(built, tmp_path, preset, seed):
    errs = gen_check.check(preset, seed=seed, tmpdir=str(tmp_path))
    assert not errs, "\n".join(errs)


def test_parser_matches_generator_1080p(built, tmp_path):
    errs = gen_check.check("c3", seed=11, extra=("frames=5",), tmpdir=str(tmp_path))
    assert not errs, "\n".join(errs)
