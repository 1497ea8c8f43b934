#!/usr/bin/env python3
"""Convert an ISO-BMFF/MP4 H.264 track into an Annex-B elementary stream (.264).

Used to build fixture F1 from imageio's `realshort.mp4`: the avcC SPS/PPS are
written once with 4-byte start codes, then every length-prefixed NAL of every sample in decode
order, also with 4-byte start codes.  Expected output sha256:
ab39814a226782e5488b337e521bb02b261ea3d09e3fcf2fc21078b0a58ec9de
"""
import struct
import sys

F1_MP4 = "/opt/conda/lib/python3.9/site-packages/imageio/resources/images/realshort.mp4"
F1_SHA256 = "ab39814a226782e5488b337e521bb02b261ea3d09e3fcf2fc21078b0a58ec9de"


def boxes(buf, off, end):
    while off + 8 <= end:
        size, typ = struct.unpack(">I4s", buf[off:off + 8])
        hdr = 8
        if size == 1:
            size = struct.unpack(">Q", buf[off + 8:off + 16])[0]
            hdr = 16
        elif size == 0:
            size = end - off
        yield typ.decode("latin1"), off + hdr, off + size
        off += size


def find(buf, off, end, path):
    for typ, b, e in boxes(buf, off, end):
        if typ == path[0]:
            if len(path) == 1:
                return b, e
            r = find(buf, b, e, path[1:])
            if r:
                return r
    return None


def video_trak(buf, moov):
    for typ, b, e in boxes(buf, *moov):
        if typ != "trak":
            continue
        hd = find(buf, b, e, ["mdia", "hdlr"])
        if hd and buf[hd[0] + 8:hd[0] + 12] == b"vide":
            return b, e
    raise ValueError("no video track")


def convert(data):
    moov = find(data, 0, len(data), ["moov"])
    trak = video_trak(data, moov)
    stbl = find(data, *trak, ["mdia", "minf", "stbl"])
    stsd = find(data, *stbl, ["stsd"])
    # stsd: version/flags(4) entry_count(4) then sample entries; avc1 has 78 bytes of fields
    ent = stsd[0] + 8
    esize, etype = struct.unpack(">I4s", data[ent:ent + 8])
    assert etype in (b"avc1", b"avc3"), etype
    avcc = find(data, ent + 8 + 78, ent + esize, ["avcC"])
    p = avcc[0]
    nal_len_size = (data[p + 4] & 3) + 1
    nsps = data[p + 5] & 31
    q = p + 6
    params = []
    for _ in range(nsps):
        n = struct.unpack(">H", data[q:q + 2])[0]
        params.append(data[q + 2:q + 2 + n])
        q += 2 + n
    npps = data[q]
    q += 1
    for _ in range(npps):
        n = struct.unpack(">H", data[q:q + 2])[0]
        params.append(data[q + 2:q + 2 + n])
        q += 2 + n

    def table(name):
        return find(data, *stbl, [name])

    stsz = table("stsz")
    sample_size, count = struct.unpack(">II", data[stsz[0] + 4:stsz[0] + 12])
    sizes = ([sample_size] * count if sample_size else
             list(struct.unpack(">%dI" % count, data[stsz[0] + 12:stsz[0] + 12 + 4 * count])))
    co = table("stco")
    if co:
        n = struct.unpack(">I", data[co[0] + 4:co[0] + 8])[0]
        offsets = list(struct.unpack(">%dI" % n, data[co[0] + 8:co[0] + 8 + 4 * n]))
    else:
        co = table("co64")
        n = struct.unpack(">I", data[co[0] + 4:co[0] + 8])[0]
        offsets = list(struct.unpack(">%dQ" % n, data[co[0] + 8:co[0] + 8 + 8 * n]))
    stsc = table("stsc")
    n = struct.unpack(">I", data[stsc[0] + 4:stsc[0] + 8])[0]
    runs = [struct.unpack(">III", data[stsc[0] + 8 + 12 * i:stsc[0] + 20 + 12 * i]) for i in range(n)]

    out = bytearray()
    for ps in params:
        out += b"\x00\x00\x00\x01" + ps
    si = 0
    for ci, coff in enumerate(offsets):
        chunk = ci + 1
        per = 0
        for first, spc, _ in runs:
            if chunk >= first:
                per = spc
        pos = coff
        for _ in range(per):
            if si >= len(sizes):
                break
            end = pos + sizes[si]
            while pos < end:
                ln = int.from_bytes(data[pos:pos + nal_len_size], "big")
                pos += nal_len_size
                out += b"\x00\x00\x00\x01" + data[pos:pos + ln]
                pos += ln
            si += 1
    return bytes(out)


def main(argv):
    src = argv[1] if len(argv) > 1 else F1_MP4
    dst = argv[2] if len(argv) > 2 else "realshort.264"
    data = open(src, "rb").read()
    out = convert(data)
    open(dst, "wb").write(out)
    import hashlib
    print(dst, len(out), hashlib.sha256(out).hexdigest())


if __name__ == "__main__":
    main(sys.argv)
