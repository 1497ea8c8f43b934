"""Test-only access to the CPU oracle (oracle/recon_oracle.c) as an m2r_backend_t.

The oracle is the parity checker; it is never the thing measured or shipped."""
import ctypes
import os

from m2dec_amd import Backend

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
_orc = None


def oracle_lib():
    global _orc
    if _orc is None:
        _orc = ctypes.CDLL(ORACLE_PATH)
        _orc.oracle_backend_create.argtypes = [ctypes.POINTER(Backend)]
        _orc.oracle_backend_create.restype = ctypes.c_int
        _orc.oracle_domain_violations.argtypes = [ctypes.c_int]
        _orc.oracle_domain_violations.restype = ctypes.c_ulong
        _orc.oracle_quirk_hits.argtypes = [ctypes.c_int, ctypes.c_int]
        _orc.oracle_quirk_hits.restype = ctypes.c_ulong
    return _orc


def domain_violations(reset=True):
    """CLIP255C arguments outside the reference table's domain since the last reset (Appendix A #2)."""
    return int(oracle_lib().oracle_domain_violations(1 if reset else 0))


class OracleBackend:
    def __init__(self):
        self.be = Backend()
        assert oracle_lib().oracle_backend_create(ctypes.byref(self.be)) == 0

    def close(self):
        if self.be.destroy:
            ctypes.CFUNCTYPE(None, ctypes.c_void_p)(self.be.destroy)(self.be.self)
            self.be.destroy = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def golden_md5s(path):
    data = open(path, "rb").read()
    assert len(data) % 34 == 0
    return [data[i:i + 32].decode() for i in range(0, len(data), 34)]


QUIRKS = ["sat16", "w128_explicit", "w128_implicit", "swar_big", "deq8_trunc", "umv", "pcm", "swar_calls"]


def quirk_hits(reset=True):
    """Counts of the Appendix A quirk paths the oracle executed since the last reset (recon_oracle.c)."""
    return {q: int(oracle_lib().oracle_quirk_hits(i, 1 if reset else 0)) for i, q in enumerate(QUIRKS)}


# ---- H.265: oracle/h265_oracle.c as an h265r_backend_t
def _h265_lib():
    L = oracle_lib()
    from m2dec_amd import Backend265
    L.h265_oracle_backend_create.argtypes = [ctypes.POINTER(Backend265)]
    L.h265_oracle_backend_create.restype = ctypes.c_int
    L.h265_oracle_violations.argtypes = [ctypes.c_int]
    L.h265_oracle_violations.restype = ctypes.c_uint64
    return L


def h265_violations(reset=True):
    """CLIP255C arguments outside [-256, 767] and DC-only terms beyond the SWAR byte range seen by the H.265
    oracle since the last reset."""
    return int(_h265_lib().h265_oracle_violations(1 if reset else 0))


class Oracle265Backend:
    def __init__(self):
        from m2dec_amd import Backend265
        self.be = Backend265()
        assert _h265_lib().h265_oracle_backend_create(ctypes.byref(self.be)) == 0

    def close(self):
        if self.be.destroy:
            ctypes.CFUNCTYPE(None, ctypes.c_void_p)(self.be.destroy)(self.be.self)
            self.be.destroy = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
