"""Interchange formats, host side: bincode HnswState
(index/hnsw.rs:47-226), hnsw_rs dump description (hnswio.rs:878-1040),
feature-file headers (mmap.rs:147-218, cold_tier.rs:17-151). No GPU needed.

Parity: bincode 2.0.1 is not vendored under the reference; its standard
config (little-endian, varint: <251 one byte, 251/252/253 + u16/u32/u64) is
restated from the published crate and pinned by the hand-derived byte strings
below. The hnsw_rs format is pinned by its vendored source (tests/hnswrs_io.py)."""
import os
import struct

import numpy as np
import pytest

import hnswrs_io as H
import oracle as O
from ruvector_amd import formats as F


def test_bincode_varint_golden():
    assert F.enc_varint(0) == b"\x00" and F.enc_varint(250) == b"\xfa"
    assert F.enc_varint(251) == b"\xfb\xfb\x00"
    assert F.enc_varint(65535) == b"\xfb\xff\xff"
    assert F.enc_varint(65536) == b"\xfc\x00\x00\x01\x00"
    assert F.enc_varint(1 << 32) == b"\xfd" + (1 << 32).to_bytes(8, "little")


def test_hnsw_state_golden_bytes_and_round_trip():
    st = F.HnswState(vectors=[("a", np.array([1.0, -2.0], np.float32))], id_to_idx=[("a", 0)], idx_to_id=[(0, "a")],
                     next_idx=1, m=32, ef_construction=200, ef_search=100, max_elements=10_000_000, dimensions=2,
                     metric="Cosine")
    b = st.encode()
    expect = (b"\x01" + b"\x01a" + b"\x02" + struct.pack("<ff", 1.0, -2.0)  # vectors
              + b"\x01" + b"\x01a\x00"                                        # id_to_idx
              + b"\x01" + b"\x00\x01a"                                        # idx_to_id
              + b"\x01"                                                       # next_idx
              + b"\x20" + b"\xc8" + b"\x64" + b"\xfc" + struct.pack("<I", 10_000_000)  # config
              + b"\x02" + b"\x01")                                            # dimensions, metric
    assert b == expect
    back = F.HnswState.decode(b)
    assert back.metric == "Cosine" and back.next_idx == 1 and back.max_elements == 10_000_000
    assert back.vectors[0][0] == "a" and np.array_equal(back.vectors[0][1], [1.0, -2.0])
    with pytest.raises(Exception):
        F.HnswState.decode(b[:-3])


def test_hnswrs_dump_description(tmp_path):
    n, d = 300, 16
    x = O.fill_uniform(n * d, 3).reshape(n, d)
    h = O.Hnsw(d, "l2", m=8, ef_construction=40, seed=3)
    h.insert(x, threads=4)
    ids = np.arange(1000, 1000 + n, dtype=np.uint64)
    base = str(tmp_path / "idx")
    H.write_dump(base, h.export(), x, ids, 8, 40)
    ds = F.describe_dump(str(tmp_path), "idx")
    assert ds["format_version"] == 4 and ds["dump_mode"] == 1 and ds["max_nb_connection"] == 8
    assert ds["nb_layer"] == 16 and ds["ef"] == 40 and ds["nb_point"] == n and ds["dimension"] == d
    assert ds["distname"].endswith("DistL2") and ds["t_name"] == "f32"
    back = H.read_dump(base)  # the test-side reader agrees with the writer
    assert len(back["points"]) == n and np.array_equal(back["vectors"][1005], x[5])


def test_feature_file_headers(tmp_path):
    d, n = 12, 7
    x = np.arange(n * d, dtype=np.float32).reshape(n, d)
    raw = str(tmp_path / "emb.bin")
    x.tofile(raw)
    assert F.feature_file_info(raw, F.RAW, d) == {"rows": n, "dim": d, "block_size": 4 * d}
    cold = str(tmp_path / "feat.cold")
    with open(cold, "wb") as f:
        f.write(struct.pack("<QQQ", d, n, 4096))
        for r in x:
            f.write(r.tobytes() + b"\0" * (4096 - 4 * d))
    assert F.feature_file_info(cold, F.COLD_TIER) == {"rows": n, "dim": d, "block_size": 4096}
    from ruvector_amd import RvxError
    with pytest.raises(RvxError):
        F.feature_file_info(cold, F.COLD_TIER, d + 1)
    with pytest.raises(RvxError):
        F.feature_file_info(str(tmp_path / "missing"), F.RAW, d)
