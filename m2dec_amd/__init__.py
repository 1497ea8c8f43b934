"""m2dec_amd — MI355X (gfx950) macroblock-reconstruction back end for the m2dec H.264 decoder.

Host-side mirror of the reference's decoder API (``m2d_func_table_t h264d_func``,
/root/reference/src/lib/m2d.h:66-75, h264.cpp:12057-12068) and of its stream driver
(src/app/h264dec.cpp + m2decoder.h), bound over ctypes to ``m2dec_amd/lib/libm2dec_amd.so``.

The product path is: host C parser (CABAC/CAVLC/MV/DPB) -> per-picture records (include/m2d_recon.h)
-> hand-written HIP kernels (m2dec_amd/csrc/hip/recon_hip.hip) -> NV12 frames in the caller's host
buffers.  There is no CPU reconstruction in this package: ``decode_stream`` without an explicit
back end uses the HIP back end and raises if no gfx950 device is usable.
"""
from __future__ import annotations

import ctypes
import os
from typing import Callable, List, Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("M2DEC_AMD_LIB") or os.path.join(_HERE, "lib", "libm2dec_amd.so")

__all__ = [
    "LIB_PATH", "Frame", "Backend", "Stats", "HipTiming", "lib", "hip_available", "HipBackend",
    "decode_stream", "decode_stream_md5", "decode_streams", "decode_m2v", "m2v_last_checks", "decode_table_frames", "frame_md5", "frame_nv12", "H264Decoder", "Trace", "HipReplay", "TracePic",
]


class Frame(ctypes.Structure):
    """m2d_frame_t (reference m2d.h:35-42)."""
    _fields_ = [("luma", ctypes.c_void_p), ("chroma", ctypes.c_void_p), ("id", ctypes.c_void_p),
                ("cnt", ctypes.c_int32), ("width", ctypes.c_int16), ("height", ctypes.c_int16),
                ("crop", ctypes.c_int16 * 4)]


class Info(ctypes.Structure):
    """m2d_info_t (reference m2d.h:44-50)."""
    _fields_ = [("src_width", ctypes.c_int16), ("src_height", ctypes.c_int16), ("disp_width", ctypes.c_int16),
                ("disp_height", ctypes.c_int16), ("frame_num", ctypes.c_int16), ("crop", ctypes.c_int16 * 4),
                ("additional_size", ctypes.c_int)]


class Backend(ctypes.Structure):
    """m2r_backend_t (include/m2d_recon.h): self + set_frames/acquire/submit/sync_frame/destroy/bind/flush/ready/
    records_busy."""
    _fields_ = [("self", ctypes.c_void_p), ("set_frames", ctypes.c_void_p), ("acquire", ctypes.c_void_p),
                ("submit", ctypes.c_void_p), ("sync_frame", ctypes.c_void_p), ("destroy", ctypes.c_void_p),
                ("bind", ctypes.c_void_p), ("flush", ctypes.c_void_p), ("ready", ctypes.c_void_p),
                ("records_busy", ctypes.c_void_p)]


class Stats(ctypes.Structure):
    """m2dec_amd_stats_t (include/m2dec_amd.h)."""
    _fields_ = [("frames_out", ctypes.c_int), ("pictures", ctypes.c_int), ("last_error", ctypes.c_int),
                ("ahead", ctypes.c_int), ("t_start", ctypes.c_double), ("t_end", ctypes.c_double),
                ("setup_s", ctypes.c_double), ("kernel_us", ctypes.c_double), ("kernel_launches", ctypes.c_int64),
                ("alg_bytes", ctypes.c_int64), ("hold_waits", ctypes.c_int64),
                ("h2d_us", ctypes.c_double), ("d2h_us", ctypes.c_double), ("parse_cpu_s", ctypes.c_double),
                ("slice_par_pictures", ctypes.c_int64), ("slice_par_fallbacks", ctypes.c_int64),
                ("teardown_s", ctypes.c_double), ("d2h_bytes", ctypes.c_int64), ("host_copy_us", ctypes.c_double)]


class HipTiming(ctypes.Structure):
    """m2dec_amd_hip_timing_t (include/m2dec_amd.h)."""
    _fields_ = [("picture_us", ctypes.c_double), ("h2d_us", ctypes.c_double), ("d2h_us", ctypes.c_double),
                ("pictures", ctypes.c_int64),
                ("inter_launches", ctypes.c_int64), ("intra_launches", ctypes.c_int64),
                ("deblock_launches", ctypes.c_int64), ("record_bytes", ctypes.c_int64),
                ("ref_bytes", ctypes.c_int64), ("frame_bytes", ctypes.c_int64), ("kernel_launches", ctypes.c_int64),
                ("d2h_bytes", ctypes.c_int64), ("host_copy_us", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class HipBudget(ctypes.Structure):
    """m2dec_amd_hip_budget_t (include/m2dec_amd.h)."""
    _fields_ = [(k, ctypes.c_int) for k in ("resident_per_cu", "cap_workgroups", "wg_units", "cap_units", "pics_fit",
                                            "launch_limit", "streams", "shared", "max_procs", "max_units")]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class TracePic(ctypes.Structure):
    """m2dec_amd_trace_pic_t (include/m2dec_amd.h)."""
    _fields_ = [("slot", ctypes.c_int32), ("width_mbs", ctypes.c_int32), ("height_mbs", ctypes.c_int32),
                ("n_inter", ctypes.c_int32), ("n_coef", ctypes.c_int32), ("n_slices", ctypes.c_int32),
                ("n_intra", ctypes.c_int32), ("deblock", ctypes.c_int32), ("off_mb", ctypes.c_uint64),
                ("off_dbk", ctypes.c_uint64), ("off_slice", ctypes.c_uint64), ("off_inter", ctypes.c_uint64),
                ("off_coef", ctypes.c_uint64), ("record_bytes", ctypes.c_int64), ("ref_bytes", ctypes.c_int64),
                ("frame_bytes", ctypes.c_int64)]


ON_FRAME = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(Frame))

_lib = None


def lib() -> ctypes.CDLL:
    """Load libm2dec_amd.so (built in-tree by ``make`` / ``__graft_entry__.build()``)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"m2dec_amd: {LIB_PATH} is not built (run `make` or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        L.m2dec_amd_decode_stream.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(Backend), ctypes.c_int,
                                              ON_FRAME, ctypes.c_void_p, ctypes.POINTER(Stats)]
        L.m2dec_amd_decode_stream.restype = ctypes.c_int
        L.m2dec_amd_decode_stream3.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(Backend), ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ON_FRAME, ctypes.c_void_p,
                                               ctypes.POINTER(Stats)]
        L.m2dec_amd_decode_stream3.restype = ctypes.c_int
        L.m2dec_amd_hip_backend_create.argtypes = [ctypes.POINTER(Backend), ctypes.c_int]
        L.m2dec_amd_hip_backend_create.restype = ctypes.c_int
        L.m2dec_amd_hip_available.argtypes = []
        L.m2dec_amd_hip_available.restype = ctypes.c_int
        L.m2dec_amd_hip_backend_timing.argtypes = [ctypes.POINTER(Backend), ctypes.POINTER(HipTiming)]
        L.m2dec_amd_hip_backend_timing.restype = ctypes.c_int
        L.m2dec_amd_hip_backend_budget.argtypes = [ctypes.POINTER(Backend), ctypes.POINTER(HipBudget)]
        L.m2dec_amd_hip_backend_budget.restype = ctypes.c_int
        L.m2dec_amd_pinned_bytes.argtypes = [ctypes.POINTER(ctypes.c_longlong)]
        L.m2dec_amd_pinned_bytes.restype = ctypes.c_longlong
        L.m2dec_amd_release_pools.argtypes = []
        L.m2dec_amd_release_pools.restype = None
        L.m2dec_amd_frame_md5.argtypes = [ctypes.POINTER(Frame), ctypes.c_char_p]
        L.m2dec_amd_frame_md5.restype = None
        L.m2dec_amd_frames_md5.argtypes = [ctypes.POINTER(Frame), ctypes.c_int, ctypes.c_char_p]
        L.m2dec_amd_frames_md5.restype = ctypes.c_int
        L.m2dec_amd_decode_stream_md5.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(Stats)]
        L.m2dec_amd_decode_stream_md5.restype = ctypes.c_int
        L.m2dec_amd_decode_stream_md5_backend.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(Backend),
                                                          ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                                          ctypes.POINTER(Stats)]
        L.m2dec_amd_decode_stream_md5_backend.restype = ctypes.c_int
        L.m2dec_amd_decode_streams_md5.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                                   ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                                   ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_int),
                                                   ctypes.POINTER(ctypes.c_int)]
        L.m2dec_amd_decode_streams_md5.restype = ctypes.c_int
        vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
        L.m2dec_amd_trace_capture.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp)]
        L.m2dec_amd_trace_capture.restype = ctypes.c_int
        L.m2dec_amd_trace_info.argtypes = [vp, ip, ip, ip, ip, ip]
        L.m2dec_amd_trace_info.restype = ctypes.c_int
        L.m2dec_amd_trace_pictures.argtypes = [vp]
        L.m2dec_amd_trace_pictures.restype = ctypes.POINTER(TracePic)
        L.m2dec_amd_trace_records.argtypes = [vp, ctypes.POINTER(ctypes.c_size_t)]
        L.m2dec_amd_trace_records.restype = vp
        L.m2dec_amd_trace_output_order.argtypes = [vp]
        L.m2dec_amd_trace_output_order.restype = ip
        L.m2dec_amd_trace_crop.argtypes = [vp, ip]
        L.m2dec_amd_trace_crop.restype = ctypes.c_int
        L.m2dec_amd_trace_free.argtypes = [vp]
        L.m2dec_amd_trace_free.restype = None
        L.m2dec_amd_hip_replay_create.argtypes = [vp, ctypes.c_int, ctypes.POINTER(vp)]
        L.m2dec_amd_hip_replay_create.restype = ctypes.c_int
        L.m2dec_amd_hip_replay_create_multi.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        L.m2dec_amd_hip_replay_create_multi.restype = ctypes.c_int
        L.m2dec_amd_hip_replay_stream.argtypes = [vp, ctypes.c_int]
        L.m2dec_amd_hip_replay_stream.restype = ctypes.c_int
        L.m2dec_amd_hip_replay_run.argtypes = [vp, ctypes.c_int]
        L.m2dec_amd_hip_replay_run.restype = ctypes.c_int
        L.m2dec_amd_hip_replay_sync.argtypes = [vp]
        L.m2dec_amd_hip_replay_sync.restype = ctypes.c_int
        L.m2dec_amd_hip_replay_timing.argtypes = [vp, ctypes.POINTER(HipTiming), ctypes.c_int]
        L.m2dec_amd_hip_replay_timing.restype = ctypes.c_int
        L.m2dec_amd_hip_replay_md5.argtypes = [vp, ctypes.c_char_p]
        L.m2dec_amd_hip_replay_md5.restype = ctypes.c_int
        L.m2dec_amd_hip_replay_capture.argtypes = [vp, ctypes.c_void_p, ctypes.c_size_t]
        L.m2dec_amd_hip_replay_capture.restype = ctypes.c_int
        L.m2dec_amd_decode_table.argtypes = [vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ON_FRAME, vp, ctypes.POINTER(ctypes.c_int)]
        L.m2dec_amd_decode_table.restype = ctypes.c_int
        L.m2dec_amd_decode_table2.argtypes = [vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.POINTER(Backend), ctypes.c_int, ON_FRAME,
                                              vp, ctypes.POINTER(ctypes.c_int)]
        L.m2dec_amd_decode_table2.restype = ctypes.c_int
        L.m2dec_amd_decode_m2v.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ON_FRAME, vp,
                                           ctypes.POINTER(ctypes.c_int)]
        L.m2dec_amd_decode_m2v.restype = ctypes.c_int
        L.m2dec_amd_m2v_dct_code.argtypes = [ctypes.c_int, ctypes.c_uint32, ip, ip]
        L.m2dec_amd_m2v_vlc_code.argtypes = [ctypes.c_int, ctypes.c_uint32, ip]
        L.m2dec_amd_m2v_intra_dc.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ip]
        L.m2dec_amd_m2v_intra_ac.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_int16)]
        L.m2dec_amd_hip_replay_destroy.argtypes = [vp]
        L.m2dec_amd_hip_replay_destroy.restype = None
        _lib = L
    return _lib


def cpu_gate() -> dict:
    """The host CPU share this process runs with (cpushare.c): share, busy-thread slots (= parse pool), how
    often an MD5 batch waited for a free slot, and the parse / MD5 work running now."""
    L = lib()
    sl, pr, bu = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    w = ctypes.c_ulong()
    L.m2dec_amd_cpu_gate.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_ulong),
                                     ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    share = L.m2dec_amd_cpu_gate(ctypes.byref(sl), ctypes.byref(w), ctypes.byref(pr), ctypes.byref(bu))
    return {"share": share, "slots": sl.value, "md5_waits": w.value, "parse_now": pr.value, "md5_now": bu.value}


def hip_available() -> bool:
    return bool(lib().m2dec_amd_hip_available())


def _call_destroy(be: Backend) -> None:
    if be.destroy:
        ctypes.CFUNCTYPE(None, ctypes.c_void_p)(be.destroy)(be.self)
        be.destroy = None


class HipBackend:
    """The gfx950 reconstruction back end (m2dec_amd_hip_backend_create).  Raises if unavailable."""

    def __init__(self, device: int = 0):
        self.be = Backend()
        if lib().m2dec_amd_hip_backend_create(ctypes.byref(self.be), device) < 0:
            raise RuntimeError(f"m2dec_amd: HIP back end unavailable on device {device} (needs a gfx950 GPU)")

    def timing(self) -> dict:
        t = HipTiming()
        lib().m2dec_amd_hip_backend_timing(ctypes.byref(self.be), ctypes.byref(t))
        return t.as_dict()

    def budget(self) -> dict:
        """What this context plans with against the device-wide workgroup budget (m2dec_amd_hip_backend_budget)."""
        b = HipBudget()
        lib().m2dec_amd_hip_backend_budget(ctypes.byref(self.be), ctypes.byref(b))
        return b.as_dict()

    def close(self) -> None:
        _call_destroy(self.be)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def frame_md5(f: Frame) -> str:
    """FileWriterMd5 line for one frame (reference filewrite.h:99-124), without the CRLF."""
    buf = ctypes.create_string_buffer(35)
    lib().m2dec_amd_frame_md5(ctypes.byref(f), buf)
    return buf.raw[:32].decode()


def frame_nv12(f: Frame) -> bytes:
    """Cropped Y rows then cropped interleaved CbCr rows (FileWriter, filewrite.h:11-29)."""
    w, h = f.width, f.height
    l, r, t, b = f.crop[0], f.crop[1], f.crop[2], f.crop[3]
    out = bytearray()
    luma = ctypes.cast(f.luma, ctypes.POINTER(ctypes.c_uint8))
    chroma = ctypes.cast(f.chroma, ctypes.POINTER(ctypes.c_uint8))
    for y in range(t, h - b):
        out += ctypes.string_at(ctypes.addressof(luma.contents) + y * w + l, w - l - r)
    for y in range(t // 2, (h - b) // 2):
        out += ctypes.string_at(ctypes.addressof(chroma.contents) + y * w + l, w - l - r)
    return bytes(out)


def decode_stream(data: bytes, backend: Optional[Backend] = None, device: int = 0,
                  on_frame: Optional[Callable[[Frame], None]] = None, md5: bool = True,
                  parse_threads: int = -1, stats: Optional[Stats] = None) -> List[str]:
    """Decode an Annex-B H.264 stream exactly like ``h264dec -O`` and return the per-frame MD5 list.

    ``backend`` None -> the HIP back end on ``device`` (raises if absent).  Any other m2r_backend_t
    (e.g. the oracle's, in tests) is borrowed.  ``parse_threads``: parse-ahead workers (-1: the
    default — 16 with the HIP back end, none with a borrowed one).  ``stats`` (a Stats) receives the
    decoder's counters.
    """
    L = lib()
    if backend is None and not L.m2dec_amd_hip_available():
        raise RuntimeError("m2dec_amd: no usable gfx950 device for the HIP back end")
    md5s: List[str] = []
    errs: List[BaseException] = []

    def _cb(_arg, fp):
        try:
            f = fp.contents
            if md5:
                md5s.append(frame_md5(f))
            if on_frame is not None:
                on_frame(f)
        except BaseException as e:  # noqa: BLE001 - re-raised after the C call returns
            errs.append(e)

    cb = ON_FRAME(_cb)
    st = stats if stats is not None else Stats()
    n = L.m2dec_amd_decode_stream3(data, len(data), ctypes.byref(backend) if backend is not None else None, device, -1,
                                   parse_threads, cb, None, ctypes.byref(st))
    if errs:
        raise errs[0]
    if n < 0:
        raise RuntimeError(f"m2dec_amd: decode failed (last_error={st.last_error}, frames={st.frames_out})")
    return md5s


def _max_frames(data: bytes) -> int:
    """Upper bound on output frames: one per slice NAL start code (never fewer than pictures)."""
    return max(1, data.count(b"\x00\x00\x01"))


def decode_stream_md5(data: bytes, device: int = 0, dpb: int = -1, stats: Optional[Stats] = None) -> List[str]:
    """The HIP decode path exactly like ``h264dec -O`` (``-d dpb``) with the MD5s computed in C on helper
    threads (m2dec_amd_decode_stream_md5): the throughput form of ``decode_stream``.  ``stats`` (a
    Stats) receives the §8d interval: first decode_picture -> last MD5 line written (t_start, t_end)."""
    L = lib()
    if not L.m2dec_amd_hip_available():
        raise RuntimeError("m2dec_amd: no usable gfx950 device for the HIP back end")
    cap = _max_frames(data)
    buf = ctypes.create_string_buffer(35 * cap)
    st = stats if stats is not None else Stats()
    n = L.m2dec_amd_decode_stream_md5(data, len(data), device, dpb, buf, cap, ctypes.byref(st))
    if n < 0:
        raise RuntimeError(f"m2dec_amd: decode failed (last_error={st.last_error}, frames={st.frames_out})")
    raw = buf.raw
    return [raw[35 * i:35 * i + 32].decode() for i in range(min(n, cap))]


def decode_stream_md5_backend(data: bytes, backend: Backend, parse_threads: int = 4, md5_threads: int = 2,
                              stats: Optional[Stats] = None) -> List[str]:
    """``decode_stream_md5``'s driver (frames held while helper threads hash them in place, 16 at a
    time) over a borrowed back end — the CPU oracle in tests."""
    cap = _max_frames(data)
    buf = ctypes.create_string_buffer(35 * cap)
    st = stats if stats is not None else Stats()
    n = lib().m2dec_amd_decode_stream_md5_backend(data, len(data), ctypes.byref(backend), parse_threads, md5_threads,
                                                  buf, cap, ctypes.byref(st))
    if n < 0:
        raise RuntimeError(f"m2dec_amd: decode failed (last_error={st.last_error}, frames={st.frames_out})")
    raw = buf.raw
    return [raw[35 * i:35 * i + 32].decode() for i in range(min(n, cap))]


def decode_streams(datas: List[bytes], device: int = 0) -> List[List[str]]:
    """Independent streams decoded concurrently on one device, one host thread and decoder context
    each (m2dec_amd_decode_streams_md5); per-stream MD5 lists."""
    L = lib()
    if not L.m2dec_amd_hip_available():
        raise RuntimeError("m2dec_amd: no usable gfx950 device for the HIP back end")
    n = len(datas)
    caps = [_max_frames(d) for d in datas]
    bufs = [ctypes.create_string_buffer(35 * c) for c in caps]
    arr_d = (ctypes.c_char_p * n)(*datas)
    arr_l = (ctypes.c_size_t * n)(*[len(d) for d in datas])
    arr_m = (ctypes.c_char_p * n)(*[ctypes.cast(b, ctypes.c_char_p) for b in bufs])
    arr_c = (ctypes.c_int * n)(*caps)
    frames = (ctypes.c_int * n)()
    r = L.m2dec_amd_decode_streams_md5(n, arr_d, arr_l, device, arr_m, arr_c, frames)
    if r < 0:
        raise RuntimeError(f"m2dec_amd: multi-stream decode failed (frames {list(frames)})")
    out = []
    for i in range(n):
        raw = bufs[i].raw
        out.append([raw[35 * k:35 * k + 32].decode() for k in range(min(frames[i], caps[i]))])
    return out


def decode_table_frames(table: str, data: bytes, dpb: int = -1, emptify: bool = False, skip: int = 0,
                        on_frame: Optional[Callable[[Frame], None]] = None, backend: Optional[Backend] = None,
                        parse_threads: int = -1) -> tuple:
    """M2Decoder over the reference-shaped function table ``table`` ("m2d_func" MPEG-1/2 on the CPU, or
    "h264d_func") exactly like the ``h264dec`` CLI (m2dec_amd_decode_table): returns (MD5 lines,
    last decode_picture result: -2 end of data / -1 error)."""
    L = lib()
    md5s: List[str] = []

    def _cb(_arg, fp):
        md5s.append(frame_md5(fp.contents))
        if on_frame is not None:
            on_frame(fp.contents)

    cb = ON_FRAME(_cb)
    err = ctypes.c_int()
    tab = ctypes.c_void_p.in_dll(L, table)
    L.m2dec_amd_decode_table2(tab, 1 if table == "h264d_func" else 0, data, len(data), dpb, int(emptify), skip,
                              ctypes.byref(backend) if backend is not None else None, parse_threads, cb, None,
                              ctypes.byref(err))
    return md5s, err.value


def m2v_last_checks() -> tuple:
    """(CLIP255C arguments outside the reference table's domain, motion-compensated reads outside the
    reference frame) of this thread's last MPEG-2 decode — both 0 for a stream whose output does not
    depend on reference undefined behaviour (host reconstruction only)."""
    L = lib()
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    L.m2dec_amd_m2v_last_checks(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def decode_m2v(data: bytes, device: Optional[int] = None, emptify: bool = False) -> List[str]:
    """An MPEG-1/2 video elementary stream through m2d_func like ``h264dec -O x.m2v``: the MD5 line of
    every output frame.  device None: host reconstruction (BASELINE.json configs[0]); else the pictures
    are reconstructed on that gfx950 device (m2dec_amd/csrc/hip/m2v_hip.hip) — an error, not a host
    fallback, when it is unusable."""
    if device is None:
        return decode_table_frames("m2d_func", data, emptify=emptify)[0]
    L = lib()
    md5s: List[str] = []

    def _cb(_arg, fp):
        md5s.append(frame_md5(fp.contents))

    cb = ON_FRAME(_cb)
    err = ctypes.c_int()
    r = L.m2dec_amd_decode_m2v(data, len(data), device, int(emptify), cb, None, ctypes.byref(err))
    if r == -3:
        raise RuntimeError(f"m2dec_amd: MPEG-2 decode on device {device} failed")
    return md5s


def m2v_hip_timing(reset: bool = False) -> dict:
    """Process-wide timing of the GPU MPEG-2 back end since the last reset: HIP-event time of its k_m2v
    launches, the pictures, and their SURVEY.md §8d algorithmic bytes."""
    L = lib()
    us, n, b = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
    L.m2dec_amd_m2v_hip_timing(ctypes.byref(us), ctypes.byref(n), ctypes.byref(b), int(reset))
    return {"kernel_us": us.value, "pictures": n.value, "bytes": b.value}


class H264Decoder:
    """Thin object over the reference-shaped ``h264d_func`` table for callers that drive
    decode_picture / get_decoded_frame themselves (mirrors M2Decoder, m2decoder.h:33-223)."""

    class _Table(ctypes.Structure):
        _fields_ = [("context_size", ctypes.c_size_t), ("init", ctypes.c_void_p), ("stream_pos", ctypes.c_void_p),
                    ("get_info", ctypes.c_void_p), ("set_frames", ctypes.c_void_p),
                    ("decode_picture", ctypes.c_void_p), ("peek_decoded_frame", ctypes.c_void_p),
                    ("get_decoded_frame", ctypes.c_void_p)]

    @classmethod
    def table(cls):
        p = ctypes.c_void_p.in_dll(lib(), "h264d_func")
        return ctypes.cast(p, ctypes.POINTER(cls._Table)).contents


class Trace:
    """A stream parsed once by the host parser; every picture's records kept in host memory
    (m2dec_amd_trace_capture).  Replayed on the GPU by HipReplay."""

    def __init__(self, data: bytes):
        L = lib()
        self.h = ctypes.c_void_p()
        n = L.m2dec_amd_trace_capture(data, len(data), ctypes.byref(self.h))
        if n < 0:
            raise RuntimeError("m2dec_amd: trace capture (host parse) failed")
        v = [ctypes.c_int() for _ in range(5)]
        L.m2dec_amd_trace_info(self.h, *[ctypes.byref(x) for x in v])
        self.npics, self.width, self.height, self.nslots, self.nout = [x.value for x in v]
        p = L.m2dec_amd_trace_pictures(self.h)
        self.pics = [p[i] for i in range(self.npics)]
        o = L.m2dec_amd_trace_output_order(self.h)
        self.output_order = [o[i] for i in range(self.nout)]
        ln = ctypes.c_size_t()
        self.records_ptr = L.m2dec_amd_trace_records(self.h, ctypes.byref(ln))
        self.records_len = ln.value

    def records(self) -> bytes:
        return ctypes.string_at(self.records_ptr, self.records_len)

    def close(self):
        if self.h:
            lib().m2dec_amd_trace_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class HipReplay:
    """GPU reconstruction of a Trace with its records resident in HBM (m2dec_amd_hip_replay_*).

    Given a list of Traces (independent streams of one frame size), one replay carries all of them:
    their pictures interleaved in one k_batch launch, each stream on its own frame slots."""

    def __init__(self, trace, device: int = 0):
        self.traces = list(trace) if isinstance(trace, (list, tuple)) else [trace]
        self.trace = self.traces[0]
        self.h = ctypes.c_void_p()
        hs = (ctypes.c_void_p * len(self.traces))(*[t.h.value for t in self.traces])
        if lib().m2dec_amd_hip_replay_create_multi(hs, len(self.traces), device, ctypes.byref(self.h)) < 0:
            raise RuntimeError(f"m2dec_amd: HIP replay unavailable on device {device}")
        self.npics = sum(t.npics for t in self.traces)

    def run(self, passes: int = 1) -> None:
        if lib().m2dec_amd_hip_replay_run(self.h, passes) < 0:
            raise RuntimeError("m2dec_amd: replay launch failed")

    def sync(self) -> None:
        if lib().m2dec_amd_hip_replay_sync(self.h) < 0:
            raise RuntimeError("m2dec_amd: replay failed on the device")

    def timing(self, reset: bool = True) -> dict:
        t = HipTiming()
        lib().m2dec_amd_hip_replay_timing(self.h, ctypes.byref(t), 1 if reset else 0)
        return t.as_dict()

    def md5_decode_order(self) -> List[str]:
        """Per picture in replay order (one stream: its decoding order)."""
        buf = ctypes.create_string_buffer(35 * self.npics)
        if lib().m2dec_amd_hip_replay_md5(self.h, buf) < 0:
            raise RuntimeError("m2dec_amd: replay md5 pass failed")
        raw = buf.raw
        return [raw[35 * i:35 * i + 32].decode() for i in range(self.npics)]

    def capture(self) -> bytes:
        """Raw NV12 pictures (uncropped) of one checked pass, decoding order, concatenated."""
        fb = self.trace.width * self.trace.height * 3 // 2
        buf = ctypes.create_string_buffer(fb * self.npics)
        if lib().m2dec_amd_hip_replay_capture(self.h, buf, len(buf)) < 0:
            raise RuntimeError("m2dec_amd: replay capture pass failed")
        return buf.raw

    def md5_output_order(self):
        """One stream: its frames' MD5s in output order; several: one such list per stream."""
        d = self.md5_decode_order()
        per = [[] for _ in self.traces]
        for i, m in enumerate(d):
            per[lib().m2dec_amd_hip_replay_stream(self.h, i)].append(m)
        out = [[p[i] for i in t.output_order] for p, t in zip(per, self.traces)]
        return out[0] if len(self.traces) == 1 else out

    def close(self):
        if self.h:
            lib().m2dec_amd_hip_replay_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Backend265(ctypes.Structure):
    """h265r_backend_t (include/m2d_recon.h)."""
    _fields_ = [("self", ctypes.c_void_p), ("set_frames", ctypes.c_void_p), ("submit", ctypes.c_void_p),
                ("sync_frame", ctypes.c_void_p), ("destroy", ctypes.c_void_p), ("stage", ctypes.c_void_p)]


def decode_h265(data: bytes, backend: Optional[Backend265] = None, device: int = 0, emptify: bool = False,
                on_frame: Optional[Callable[[Frame], None]] = None) -> tuple:
    """An H.265 elementary stream through h265d_func like ``h264dec -O x.265`` (M2Decoder, MODE_H265):
    returns (MD5 line of every output frame, last decode_picture result: -2 at the end of the data).
    ``backend`` None -> the gfx950 reconstruction on ``device`` (an error, not a host fallback, when it
    is unusable); a borrowed h265r_backend_t otherwise (the CPU oracle in tests)."""
    L = lib()
    md5s: List[str] = []
    errs: List[BaseException] = []

    def _cb(_arg, fp):
        try:
            md5s.append(frame_md5(fp.contents))
            if on_frame is not None:
                on_frame(fp.contents)
        except BaseException as e:  # noqa: BLE001 - re-raised after the C call returns
            errs.append(e)

    cb = ON_FRAME(_cb)
    err = ctypes.c_int()
    L.m2dec_amd_decode_h265.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(Backend265), ctypes.c_int,
                                        ctypes.c_int, ON_FRAME, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    L.m2dec_amd_decode_h265.restype = ctypes.c_int
    if backend is None and not L.m2dec_amd_hip_available():
        raise RuntimeError("m2dec_amd: no usable gfx950 device for the H.265 reconstruction")
    L.m2dec_amd_decode_h265(data, len(data), ctypes.byref(backend) if backend is not None else None, device,
                            int(emptify), cb, None, ctypes.byref(err))
    if errs:
        raise errs[0]
    return md5s, err.value


def decode_h265_md5(data: bytes, backend: Optional[Backend265] = None, device: int = 0, max_frames: int = 4096) -> tuple:
    """decode_h265 with the MD5 lines computed on the library's MD5 helper threads (16-lane batches) instead
    of in Python on the caller's thread: (MD5 line of every output frame, last decode_picture result)."""
    L = lib()
    buf = ctypes.create_string_buffer(35 * max_frames)
    err = ctypes.c_int()
    L.m2dec_amd_decode_h265_md5.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(Backend265), ctypes.c_int,
                                            ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.m2dec_amd_decode_h265_md5.restype = ctypes.c_int
    if backend is None and not L.m2dec_amd_hip_available():
        raise RuntimeError("m2dec_amd: no usable gfx950 device for the H.265 reconstruction")
    n = L.m2dec_amd_decode_h265_md5(data, len(data), ctypes.byref(backend) if backend is not None else None, device,
                                    buf, max_frames, ctypes.byref(err))
    if n < 0:
        raise RuntimeError("m2dec_amd: H.265 MD5 decode failed")
    raw = buf.raw
    return [raw[35 * i:35 * i + 32].decode() for i in range(min(n, max_frames))], err.value


def decode_m2v_md5(data: bytes, device: Optional[int] = None, max_frames: int = 4096) -> List[str]:
    """decode_m2v with the MD5 lines computed on the library's MD5 helper threads (m2dec_amd_decode_m2v_md5)."""
    L = lib()
    buf = ctypes.create_string_buffer(35 * max_frames)
    err = ctypes.c_int()
    L.m2dec_amd_decode_m2v_md5.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_int)]
    L.m2dec_amd_decode_m2v_md5.restype = ctypes.c_int
    n = L.m2dec_amd_decode_m2v_md5(data, len(data), -1 if device is None else device, buf, max_frames, ctypes.byref(err))
    if n < 0:
        raise RuntimeError(f"m2dec_amd: MPEG-2 MD5 decode on device {device} failed")
    raw = buf.raw
    return [raw[35 * i:35 * i + 32].decode() for i in range(min(n, max_frames))]


class H265HipBackend:
    """The gfx950 H.265 reconstruction (m2dec_amd_h265_hip_backend_create), borrowed by decode_h265 so that
    its device buffers outlive one stream.  Raises if unavailable."""

    def __init__(self, device: int = 0):
        L = lib()
        L.m2dec_amd_h265_hip_backend_create.argtypes = [ctypes.POINTER(Backend265), ctypes.c_int]
        L.m2dec_amd_h265_hip_backend_create.restype = ctypes.c_int
        self.be = Backend265()
        if L.m2dec_amd_h265_hip_backend_create(ctypes.byref(self.be), device) < 0:
            raise RuntimeError(f"m2dec_amd: H.265 HIP back end unavailable on device {device} (needs a gfx950 GPU)")

    def timing(self, reset: bool = False) -> dict:
        L = lib()
        i64 = ctypes.POINTER(ctypes.c_int64)
        L.m2dec_amd_h265_hip_timing.argtypes = [ctypes.POINTER(Backend265), ctypes.POINTER(ctypes.c_double), i64, i64,
                                                i64, ctypes.c_int]
        us, n, rb, fb = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        L.m2dec_amd_h265_hip_timing(ctypes.byref(self.be), ctypes.byref(us), ctypes.byref(n), ctypes.byref(rb),
                                    ctypes.byref(fb), int(reset))
        return {"kernel_us": us.value, "pictures": n.value, "record_bytes": rb.value, "frame_bytes": fb.value}

    def close(self) -> None:
        if self.be.destroy:
            ctypes.CFUNCTYPE(None, ctypes.c_void_p)(self.be.destroy)(self.be.self)
            self.be.destroy = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
