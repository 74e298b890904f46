"""Device bits of the libm restatements (ruvector_amd/csrc/libm_f32.hpp, compiled into the
HIP kernels) against the host's glibc, over all 2^32 f32 inputs.

These functions carry the reference's transcendental rounding into the GPU path:
fast_acosh's logf (every Poincaré distance, poincare.rs:259-276), log_map's atanh =
0.5 * log1pf(2x / (1 - x)) (Rust std f32::atanh) and exp_map's tanhf (poincare.rs:407-451).
tests/test_libm.py checks the same source compiled for the host.
"""
import numpy as np
import pytest

import oracle as O

rv = pytest.importorskip("ruvector_amd")
pytestmark = pytest.mark.gpu

CHUNK = 1 << 28


@pytest.mark.parametrize("fn", O.LIBM_FNS)
def test_device_libm_equals_glibc_on_every_input(fn):
    from ruvector_amd import _lib as L
    out = np.empty(CHUNK, np.float32)
    total = 0
    for start in range(0, 1 << 32, CHUNK):
        L.call("rvx_selftest_libm", O.LIBM_FNS.index(fn), start, 1, CHUNK, L.fptr(out))
        bad, first = O.libm_check(fn, start=start, count=CHUNK, dev=out)
        assert bad == 0, f"{fn}: {bad} device mismatches in [{start:#x}, +2^28), first at bits {first:#010x}"
        total += CHUNK
    assert total == 1 << 32
