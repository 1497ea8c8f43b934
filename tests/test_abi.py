"""The C-ABI libraries load and export every function include/*.h declares (no compute calls:
this runs without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"typedef struct[^;]*?\{.*?\}\s*\w+\s*;", "", src, flags=re.S)
    names = set()
    for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", src, flags=re.M):
        name = m.group(1)
        if name in ("if", "while", "for", "return", "sizeof"):
            continue
        names.add(name)
    return names


def test_all_declared_symbols_exported(built):
    lib = ctypes.CDLL(os.path.join(ROOT, "m2dec_amd", "lib", "libm2dec_amd.so"))
    missing = []
    for h in ("m2d.h", "m2dec_amd.h"):
        for name in sorted(_declared(h)):
            if not hasattr(lib, name):
                missing.append(f"{h}:{name}")
    assert not missing, missing
    # the reference's decoder table (h264.h:457) is an exported data symbol
    assert ctypes.c_void_p.in_dll(lib, "h264d_func").value
    assert ctypes.c_void_p.in_dll(lib, "m2d_func").value  # mpeg2.cpp:1811


def test_declared_symbol_scan_is_not_empty():
    names = _declared("m2dec_amd.h") | _declared("m2d.h")
    for expect in ("m2dec_amd_decode_stream", "m2dec_amd_hip_backend_create", "m2dec_amd_trace_capture",
                   "m2dec_amd_hip_replay_run", "dec_bits_open", "m2d_next_start_code"):
        assert expect in names


def test_h264d_func_table_shape(built):
    import m2dec_amd

    t = m2dec_amd.H264Decoder.table()
    assert t.context_size > 0
    for f in ("init", "stream_pos", "get_info", "set_frames", "decode_picture", "peek_decoded_frame",
              "get_decoded_frame"):
        assert getattr(t, f), f


def test_product_path_fails_loudly_without_gpu(built):
    import m2dec_amd

    if m2dec_amd.hip_available():
        return
    data = open(os.path.join(ROOT, "tests", "golden", "f1_realshort.264"), "rb").read()
    try:
        m2dec_amd.decode_stream(data)
    except RuntimeError:
        pass
    else:
        raise AssertionError("HIP product path must not fall back to a CPU reconstruction")


def test_abi_revision_and_sized_backend(built):
    """the structs changed size in revision 3; the library says which revision it is and
    accepts an older, smaller m2r_backend_t by size (its unknown `bind` taken as NULL)."""
    lib = ctypes.CDLL(os.path.join(ROOT, "m2dec_amd", "lib", "libm2dec_amd.so"))
    hdr = open(os.path.join(ROOT, "include", "m2dec_amd.h")).read()
    rev = int(re.search(r"#define M2DEC_AMD_ABI_VERSION (\d+)", hdr).group(1))
    assert lib.m2dec_amd_abi_version() == rev
    lib.m2dec_amd_stats_size.restype = ctypes.c_size_t
    assert lib.m2dec_amd_stats_size() >= 112
    assert lib.m2dec_amd_host_cpu_ok() == 1
    import m2dec_amd

    t = m2dec_amd.H264Decoder.table()
    ctx = ctypes.create_string_buffer(t.context_size)
    init = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)(t.init)
    assert init(ctx, -1, None, None) == 0
    be = (ctypes.c_void_p * 10)()  # self + 9 function pointers (revision 6)
    lib.m2dec_amd_h264_set_backend2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    ptr = ctypes.sizeof(ctypes.c_void_p)
    assert lib.m2dec_amd_h264_set_backend2(ctx, be, 3 * ptr) == -1   # shorter than any revision
    assert lib.m2dec_amd_h264_set_backend2(ctx, be, 11 * ptr) == -1  # longer than this revision
    assert lib.m2dec_amd_h264_set_backend2(ctx, be, 9 * ptr) == 0    # revision 5: no records_busy
    assert lib.m2dec_amd_h264_set_backend2(ctx, be, 8 * ptr) == 0    # revision 4: no ready
    assert lib.m2dec_amd_h264_set_backend2(ctx, be, 6 * ptr) == 0    # revision 2: no bind
    assert lib.m2dec_amd_h264_set_backend2(ctx, be, 7 * ptr) == 0    # revision 3: no flush
    assert lib.m2dec_amd_h264_set_backend2(ctx, None, 0) == 0        # detach (borrowed, not destroyed)
    lib.m2dec_amd_h264_release(ctx)
