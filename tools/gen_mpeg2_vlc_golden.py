"""Make tests/golden/mpeg2_vlc.json: every codeword of the reference's MPEG-2 VLC tables with the value
the reference's decoder derives from it — the golden the MPEG-2 path's own tables are tested against.

The reference's tables (/root/reference/src/lib/vld.h, "generated from standard document") are read as
text and walked exactly the way the reference's decoder walks them:
  * DCT coefficients (Tables B.14 / B.15): the inner loop of parse_coef (mpeg2.cpp:1021-1063):
    7-bit first look-up, `length <= 0` entries chain to a sub-table at +run with `level` more bits;
    run >= 0: (run, level) with the sign folded into the level's LSB; run < 0, level != 0: end of
    block; run < 0, level == 0: escape;
  * vlc_t tables (macroblock_address_increment B.1 after its leading 0 bit, dct_dc_size B.12 / B.13,
    motion_code B.10, coded_block_pattern B.9, P / B macroblock_type B.3 / B.4): m2d_dec_vld_unary
    (m2d.cpp:31-55).
Every bit string of up to 18 bits is decoded; each distinct consumed prefix is one codeword.
Only data goes into the fixture (codeword bits -> decoded value); no reference source is copied.
Run here, where /root/reference exists; the fixture is committed and the tests read only it.
"""
import json
import os
import re

REF = "/root/reference/src/lib/vld.h"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "mpeg2_vlc.json")


def tables(text):
    out = {}
    for m in re.finditer(r"static const (vlc_dct_t|vlc_t) (\w+)\[(\d+)\] = \{(.*?)\n\};", text, re.S):
        kind, name, n, body = m.group(1), m.group(2), int(m.group(3)), m.group(4)
        ent = [tuple(int(x) for x in e.split(",")) for e in re.findall(r"\{\s*(-?\d+\s*,\s*-?\d+(?:\s*,\s*-?\d+)?)\s*\}", body)]
        assert len(ent) == n, (name, len(ent), n)
        out[name] = (kind, ent)
    return out


class Bits:
    def __init__(self, s):
        self.s, self.p = s, 0

    def show(self, n):
        t = self.s[self.p:self.p + n].ljust(n, "0")
        return int(t, 2) if n else 0

    def skip(self, n):
        self.p += n


def walk_dct(tab, bits, bitlen=7):
    """parse_coef's look-up of one symbol: (consumed bits, run, level) or None (undefined code)."""
    b = Bits(bits)
    base, rest = 0, bitlen
    run, level, length = tab[base + b.show(rest)]
    while length <= 0:
        if length < 0:
            return None
        base += run
        b.skip(rest)
        rest = min(level, bitlen)
        run, level, length = tab[base + b.show(rest)]
    b.skip(length)
    return b.p, run, level


def walk_unary(tab, bits, bitlen):
    """m2d_dec_vld_unary: (consumed bits, pattern) or None (invalid code)."""
    b = Bits(bits)
    pattern, length = tab[b.show(bitlen)]
    idx = 0
    while length <= 0:
        if length == 0:
            return None
        b.skip(bitlen)
        rest = min(-length, bitlen)
        idx += pattern
        i = b.show(rest) + idx
        if i >= len(tab):
            return None
        pattern, length = tab[i]
    b.skip(length)
    return b.p, pattern


def enumerate_codes(walk, maxlen=18):
    codes = {}
    for v in range(1 << maxlen):
        s = format(v, f"0{maxlen}b")
        r = walk(s)
        if r is None:
            continue
        n = r[0]
        if n > maxlen:
            continue
        codes.setdefault(s[:n], list(r[1:]))
    # keep only codewords no other codeword is a prefix of (a walk may see an all-zero tail)
    return sorted([[k] + v for k, v in codes.items()], key=lambda x: (len(x[0]), x[0]))


def main():
    t = tables(open(REF).read())
    res = {"source": "reference vld.h tables walked as parse_coef / m2d_dec_vld_unary do (tools/gen_mpeg2_vlc_golden.py)"}
    res["dct0"] = enumerate_codes(lambda s: walk_dct(t["m2d_dct_table0_bit7"][1], s))
    res["dct1"] = enumerate_codes(lambda s: walk_dct(t["m2d_dct_table1_bit7"][1], s))
    for key, name, bl in [("mb_inc_after0", "mb_inc_bit4", 4), ("dc_luma", "dct_dc_size_luma_bit5", 5),
                          ("dc_chroma", "dct_dc_size_chroma_bit4", 4), ("motion_code", "motion_code_bit5", 5),
                          ("cbp", "coded_block_pattern_bit5", 5), ("mb_type_p", "mb_type_p_bit3", 3),
                          ("mb_type_b", "mb_type_b_bit4", 4)]:
        res[key] = enumerate_codes(lambda s, tab=t[name][1], bl=bl: walk_unary(tab, s, bl), 14)
    with open(OUT, "w") as f:
        json.dump(res, f, indent=0)
    for k, v in res.items():
        if k != "source":
            print(k, len(v))


if __name__ == "__main__":
    main()
