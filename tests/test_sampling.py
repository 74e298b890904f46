"""GraphSAGE neighbour sampling (graphsage.rs:92-102): rand 0.8.5 StdRng /
rand_chacha 0.3.1 / rand_core 0.6 restated in the oracle and in librvx.so
(host-side position tables; no GPU needed here).

Pinning: the ChaCha core is checked against RFC 7539 A.1 (the vectors of
rand_chacha's test_chacha_true_values_a) and StdRng against rand 0.8's
test_stdrng_construction value-stability targets; seed_from_u64's PCG32 fill
and partial_shuffle are restated from the published rand source (the crate is
not vendored under the reference) — the reference's own test
(graphsage.rs:237-249) pins only the sample lengths."""
import ctypes

import numpy as np
import pytest

import oracle as O


def lib_positions(length, k):
    from ruvector_amd import _lib
    out = np.empty(k, np.int32)
    _lib.call("rvx_sage_sample_positions", length, k, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return out


def test_chacha20_rfc7539_known_answer():
    w = O.chacha_words(np.zeros(8, np.uint32), 20, 32)
    assert [int(v) for v in w[:4]] == [0xade0b876, 0x903df1a0, 0xe56a5d40, 0x28bd8653]
    assert [int(v) for v in w[12:16]] == [0xf4b8436a, 0x1ca11815, 0x69b687c3, 0x8665eeb2]
    assert [int(v) for v in w[16:20]] == [0xbee7079f, 0x7a385155, 0x7c97ba98, 0x0d082d73]


def test_stdrng_value_stability():
    # rand 0.8 test_stdrng_construction: seed bytes [1,0,0,0, 23,0,0,0, 200,1,0,0, 210,30,0,0, 0...]
    w = O.chacha_words(np.array([1, 23, 456, 7890, 0, 0, 0, 0], np.uint32), 12, 10)
    x0 = int(w[1]) << 32 | int(w[0])
    w1 = O.chacha_words(w[2:10], 12, 2)  # StdRng::from_rng(rng0): next 32 bytes as the seed
    x1 = int(w1[1]) << 32 | int(w1[0])
    assert [x0, x1] == [10719222850664546238, 14064965282130556830]


def test_reference_sample_lengths():
    # graphsage.rs:237-249: 10 neighbours, k=3 -> 3; 2 neighbours, k=5 -> unchanged
    pos = O.sage_sample_positions(10, 3)
    assert len(pos) == 3 and len(set(pos.tolist())) == 3 and pos.min() >= 0 and pos.max() < 10


@pytest.mark.parametrize("length,k", [(2, 1), (10, 3), (33, 32), (64, 10), (100, 99), (1000, 25), (70000, 64),
                                      (5, 0)])
def test_library_positions_match_oracle(length, k):
    ref = O.sage_sample_positions(length, k)
    got = lib_positions(length, k)
    assert np.array_equal(got, ref)
    assert len(set(got.tolist())) == k and (k == 0 or (got.min() >= 0 and got.max() < length))


def test_library_rejects_len_le_k():
    from ruvector_amd import _lib
    with pytest.raises(_lib.RvxError):
        lib_positions(3, 3)


def test_oracle_sampled_forward_uses_sampled_subset():
    """A row with deg > k aggregates exactly the sampled neighbours, in their order."""
    n, d, k = 40, 8, 5
    x = O.fill_uniform(n * d, 7).reshape(n, d)
    rp = np.array([0, 30] + [30] * (n - 1), np.int64)  # row 0 has 30 neighbours, others none
    col = np.arange(1, 31, dtype=np.int32)
    wn, ws = O.fill_uniform(d * d, 8).reshape(d, d), O.fill_uniform(d * d, 9).reshape(d, d)
    pos = O.sage_sample_positions(30, k)
    rp_s = np.array([0, k] + [k] * (n - 1), np.int64)
    col_s = col[pos]
    y = O.sage_forward(x, rp, col, wn, ws, num_samples=k)
    y_ref = O.sage_forward(x, rp_s, col_s, wn, ws)
    assert np.array_equal(y, y_ref)
    assert np.any(y[0] != 0) and not np.array_equal(y[0], O.sage_forward(x, rp, col, wn, ws)[0])
