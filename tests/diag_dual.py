"""Diagnostic (test infrastructure): run the HIP back end and the CPU oracle side by side on the same
parsed records and report, per picture, which macroblocks differ.

    python -m tests.diag_dual stream.264 [--max-pics N]

Every picture's records go to the oracle (into shadow frames) and to the HIP back end (into the
caller's frames); after each picture the two reconstructions are compared macroblock by macroblock.
"""
import argparse
import ctypes
import sys
from collections import Counter

import numpy as np

import m2dec_amd
from m2dec_amd import Backend, Frame, HipBackend
from tests._oracle import OracleBackend

KIND = {0: "I4x4", 1: "I8x8", 2: "I16x16", 3: "PCM", 4: "INTER"}


class MB(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint8), ("cbp", ctypes.c_uint8), ("avail_luma", ctypes.c_uint8),
                ("avail_chroma", ctypes.c_uint8), ("qpy", ctypes.c_int8), ("qpc", ctypes.c_int8 * 2),
                ("pred_mode", ctypes.c_uint8), ("chroma_mode", ctypes.c_uint8), ("flags", ctypes.c_uint8),
                ("slice", ctypes.c_uint16), ("ipred", ctypes.c_uint32 * 2), ("coef", ctypes.c_uint32),
                ("nz", ctypes.c_uint32), ("inter", ctypes.c_uint32)]


class Picture(ctypes.Structure):
    _fields_ = [("width_mbs", ctypes.c_int32), ("height_mbs", ctypes.c_int32), ("slot", ctypes.c_int32),
                ("n_inter", ctypes.c_int32), ("n_coef", ctypes.c_int32), ("n_slices", ctypes.c_int32),
                ("n_intra", ctypes.c_int32), ("deblock", ctypes.c_int32), ("mb", ctypes.POINTER(MB)),
                ("dbk", ctypes.c_void_p), ("slice", ctypes.c_void_p), ("inter", ctypes.c_void_p),
                ("coef", ctypes.c_void_p), ("cap_slices", ctypes.c_int32), ("cap_inter", ctypes.c_int32),
                ("cap_coef", ctypes.c_int32), ("flags", ctypes.c_int32)]


SET_FRAMES = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Frame), ctypes.c_int,
                              ctypes.c_int)
ACQUIRE = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int)
SUBMIT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(Picture))
SYNC = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int)
DESTROY = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


def _plane(ptr, n):
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), shape=(n,))


class DualBackend:
    def __init__(self, hip: Backend, orc: Backend, verbose=True, max_report=8):
        self.hip, self.orc = hip, orc
        self.pics = 0
        self.bad = []
        self.verbose = verbose
        self.max_report = max_report
        self._cbs = [SET_FRAMES(self._set_frames), ACQUIRE(self._acquire), SUBMIT(self._submit), SYNC(self._sync),
                     DESTROY(lambda s: None)]
        self.be = Backend(None, *[ctypes.cast(c, ctypes.c_void_p).value for c in self._cbs])

    def _f(self, be, name, proto):
        return proto(getattr(be, name))

    def _set_frames(self, _s, n, frames, w, h):
        self.w, self.h, self.n = w, h, n
        self.caller = [frames[i] for i in range(n)]
        self.shadow_mem = [(np.zeros(w * h, np.uint8), np.zeros(w * h // 2, np.uint8)) for _ in range(n)]
        self.shadow = (Frame * n)()
        for i in range(n):
            self.shadow[i] = frames[i]
            self.shadow[i].luma = self.shadow_mem[i][0].ctypes.data
            self.shadow[i].chroma = self.shadow_mem[i][1].ctypes.data
        r = self._f(self.orc, "set_frames", SET_FRAMES)(self.orc.self, n, self.shadow, w, h)
        if r < 0:
            return r
        return self._f(self.hip, "set_frames", SET_FRAMES)(self.hip.self, n, frames, w, h)

    def _acquire(self, _s, wm, hm):
        return self._f(self.hip, "acquire", ACQUIRE)(self.hip.self, wm, hm)

    def _submit(self, _s, pic):
        p = pic.contents
        slot = p.slot
        r = self._f(self.orc, "submit", SUBMIT)(self.orc.self, pic)
        if r < 0:
            return r
        kinds = np.array([pic.contents.mb[i].kind for i in range(p.width_mbs * p.height_mbs)], np.uint8)
        r = self._f(self.hip, "submit", SUBMIT)(self.hip.self, pic)
        if r < 0:
            return r
        if self._f(self.hip, "sync_frame", SYNC)(self.hip.self, slot) < 0:
            print(f"pic {self.pics}: HIP sync_frame failed", file=sys.stderr)
            return -1
        self._compare(slot, kinds, p.width_mbs, p.height_mbs, p.deblock)
        self.pics += 1
        return 0

    def _sync(self, _s, slot):
        return self._f(self.hip, "sync_frame", SYNC)(self.hip.self, slot)

    def _compare(self, slot, kinds, wm, hm, deblock):
        w, h = self.w, self.h
        gy = _plane(self.caller[slot].luma, w * h).reshape(h, w)
        gc = _plane(self.caller[slot].chroma, w * h // 2).reshape(h // 2, w)
        oy = self.shadow_mem[slot][0].reshape(h, w)
        oc = self.shadow_mem[slot][1].reshape(h // 2, w)
        dy = (gy != oy).reshape(hm, 16, wm, 16).any(axis=(1, 3))
        dc = (gc != oc).reshape(hm, 8, wm, 16).any(axis=(1, 3))
        d = dy | dc
        if d.any():
            ys, xs = np.nonzero(d)
            cnt = Counter(KIND.get(int(kinds[y * wm + x]), "?") for y, x in zip(ys, xs))
            self.bad.append((self.pics, int(d.sum())))
            if self.verbose:
                print(f"pic {self.pics} slot {slot} deblock={deblock}: {int(d.sum())}/{wm * hm} MBs differ "
                      f"(luma {int(dy.sum())}, chroma {int(dc.sum())}) by kind {dict(cnt)}")
                for y, x in list(zip(ys, xs))[: self.max_report]:
                    k = KIND.get(int(kinds[y * wm + x]), "?")
                    ly = np.abs(gy[y * 16:y * 16 + 16, x * 16:x * 16 + 16].astype(int) -
                                oy[y * 16:y * 16 + 16, x * 16:x * 16 + 16]).max()
                    lc = np.abs(gc[y * 8:y * 8 + 8, x * 16:x * 16 + 16].astype(int) -
                                oc[y * 8:y * 8 + 8, x * 16:x * 16 + 16]).max()
                    print(f"   mb ({x},{y}) {k}: max |d| luma {ly} chroma {lc}")


def run(path, device=0, stop_after_first=True):
    data = open(path, "rb").read()
    with HipBackend(device) as hb, OracleBackend() as ob:
        dual = DualBackend(hb.be, ob.be)
        try:
            m2dec_amd.decode_stream(data, backend=dual.be)
        except RuntimeError as e:
            print("decode error:", e)
        return dual


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("stream")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args()
    d = run(a.stream, a.device)
    print(f"pictures {d.pics}, pictures with differences {len(d.bad)}")
    sys.exit(1 if d.bad else 0)
