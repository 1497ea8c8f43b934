"""The HIP back end's built-in known-answer test (runtime.hip m2dec_amd_hip_selftest): the
product library reconstructs two coverage streams (tools/make_selftest.py: I P B B, PCM, constrained intra,
deblocking idc 2, explicit weights) through k_batch and k_picture and matches the CPU oracle's MD5s, picture by
picture — the same check every process makes once before its first HIP back end exists."""
import ctypes
import time

import pytest

import m2dec_amd


@pytest.mark.gpu
def test_selftest_passes_on_the_product_kernels(built):
    L = m2dec_amd.lib()
    L.m2dec_amd_hip_selftest.argtypes = [ctypes.c_int]
    t0 = time.time()
    assert L.m2dec_amd_hip_selftest(0) == 0
    print(f"self-test: {1e3 * (time.time() - t0):.1f} ms")


@pytest.mark.gpu
def test_backend_creation_runs_it(built):
    with m2dec_amd.HipBackend() as be:  # (create -> selftest_once: passed, so the back end exists)
        assert be.timing() is not None
