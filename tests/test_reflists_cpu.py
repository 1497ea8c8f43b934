"""The parser's reference-picture machinery on the CPU: list modification
(h264.cpp:1608-1653), adaptive marking MMCO 1..6 and long-term pictures (:10665-11050), POC types 1 and 2
(:1159-1215), frame_num wrap, temporal direct onto a long-term picture (:10049-10054), non-reference P.

tools/h264gen restates the spec (8.2.1, 8.2.4, 8.2.5) and writes, per slice, the POC and long-term flag of
every active list entry (--dump-refs); the parser writes the same from its own lists
(m2dec_amd_h264_set_refdump), and tests/gen_check.py compares them beside every syntax element.  The
goldens (tests/golden/synthetic.json, cov_reflists* / cov_mmco5 / cov_poc*) are the oracle's frames; each
must reach the paths it was made for, counted by the parser (m2dec_amd_h264_parser_hits).  Parity
unpinned: no reference-produced output exists for these streams."""
import ctypes

import pytest

import m2dec_amd
from tests import gen_check
from tests._oracle import OracleBackend
from tests._streams import GOLDEN, stream

NAMES = ["mod0", "mod1", "mod2", "mmco1", "mmco2", "mmco3", "mmco4", "mmco5", "mmco6", "lt_list", "poc1", "poc2",
         "td_lt", "lt_idr", "fn_wrap"]

EXPECT = {
    "cov_reflists_s1": ["mod0", "mod1", "mod2", "mmco1", "mmco2", "mmco3", "mmco4", "mmco6", "lt_list", "td_lt"],
    "cov_reflists_s2": ["mod0", "mod1", "mod2", "mmco1", "mmco2", "mmco3", "lt_list", "td_lt", "lt_idr"],
    "cov_reflists_cavlc_s1": ["mod0", "mod1", "mod2", "mmco1", "mmco2", "mmco3", "mmco4", "mmco6", "lt_list"],
    "cov_mmco5_s1": ["mmco5", "mod0", "mod1"],
    "cov_poc1_s1": ["poc1"],
    "cov_poc2_s1": ["poc2", "fn_wrap", "mmco1"],
}


def hits(reset=False):
    L = m2dec_amd.lib()
    L.m2dec_amd_h264_parser_hits.argtypes = [ctypes.POINTER(ctypes.c_long), ctypes.c_int, ctypes.c_int]
    out = (ctypes.c_long * 16)()
    L.m2dec_amd_h264_parser_hits(out, 16, int(reset))
    return {n: out[i] for i, n in enumerate(NAMES)}


@pytest.mark.parametrize("name", sorted(EXPECT))
def test_golden_reaches_its_paths(built, name):
    hits(reset=True)
    with OracleBackend() as ob:
        got = m2dec_amd.decode_stream(stream(name), backend=ob.be)
    h = hits(reset=True)
    assert got == GOLDEN[name]["md5"]
    missing = [k for k in EXPECT[name] if not h[k]]
    assert not missing, (name, missing, h)


@pytest.mark.parametrize("preset,seed", [("cov_reflists", 1), ("cov_reflists", 4), ("cov_reflists_cavlc", 1),
                                         ("cov_reflists_cavlc", 5), ("cov_mmco5", 1), ("cov_mmco5", 2),
                                         ("cov_poc1", 1), ("cov_poc1", 3), ("cov_poc2", 1), ("cov_poc2", 6)])
def test_parser_lists_match_generator(built, tmp_path, preset, seed):
    """Every slice's active RefPicList0 / 1 (POC, long-term) and every MB's syntax, vectors and reference
    indices (direct blocks included) equal the generator's."""
    errs = gen_check.check(preset, seed=seed, tmpdir=str(tmp_path))
    assert not errs, errs[:10]


def test_lists_are_compared(built, tmp_path):
    """The list comparison is live: a generator list edited by one POC is reported."""
    import numpy as np

    out = str(tmp_path / "r.264")
    gen_check.generate("cov_reflists", out, seed=1, refdump=out + ".refs")
    g = np.fromfile(out + ".refs", dtype=gen_check.REFDUMP_DT)
    bad = g.copy()
    k = next(i for i in range(len(bad)) if bad[i]["n"][0] > 1)
    bad[k]["poc_l"][0][1] += 2
    assert gen_check.compare_refs(g, g) == []
    assert len(gen_check.compare_refs(bad, g)) == 1
