"""The libm restatements behind the bit-exact Poincaré path (ruvector_amd/csrc/libm_f32.hpp)
against the host's glibc 2.35, input by input over all 2^32 f32 bit patterns.

The reference calls f32::ln (glibc logf), f32::ln_1p (log1pf), f32::tanh (tanhf, through
expm1f) and std's f32::atanh = 0.5 * ln_1p(2x / (1 - x)) in fast_acosh, log_map and
exp_map (crates/ruvector-hyperbolic-hnsw/src/poincare.rs:259-276, :407-451). The same
header is compiled into the GPU kernels; tests/test_gpu_libm.py checks the device bits.
"""
import pytest

import oracle as O


@pytest.mark.parametrize("fn", O.LIBM_FNS)
def test_restatement_equals_glibc_on_every_input(fn):
    bad, first = O.libm_check(fn)
    assert bad == 0, f"{fn}: {bad} mismatches, first at bits {first:#010x}"


def test_check_counts_wrong_device_outputs():
    import numpy as np
    # x from 1.0 upwards: only log(1) = 0 is right in an all-zero "device" output
    bad, first = O.libm_check("logf", start=0x3F800000, count=4096, dev=np.zeros(4096, np.float32))
    assert bad == 4095 and first == 0x3F800001
