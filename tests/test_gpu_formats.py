"""Interchange formats on the GPU: hnsw_rs dumps loaded into / written from
the GPU index, feature files streamed into / out of HBM, HnswState
serialize/deserialize round trips."""
import struct

import numpy as np
import pytest

import hnswrs_io as H
import oracle as O

rv = pytest.importorskip("ruvector_amd")
from ruvector_amd import formats as F  # noqa: E402

pytestmark = pytest.mark.gpu


def _oracle_index(n, d, m, efc, seed, metric="l2"):
    x = O.fill_uniform(n * d, seed).reshape(n, d)
    h = O.Hnsw(d, metric, m=m, ef_construction=efc, seed=seed)
    h.insert(x, threads=8)
    return x, h


def test_load_reference_format_dump_searches_like_the_oracle(tmp_path):
    """A dump written in the reference format from the oracle's graph loads onto
    the GPU and searches bit-exactly like the oracle on that graph."""
    n, d = 3000, 32
    x, h = _oracle_index(n, d, 16, 100, 7)
    ids = np.arange(n, dtype=np.uint64) * 3 + 11  # origin ids are not row numbers
    H.write_dump(str(tmp_path / "ref"), h.export(), x, ids, 16, 100)
    ix = rv.HnswIndex.file_load(str(tmp_path), "ref")
    assert len(ix) == n and ix.metric == rv.DistanceMetric.Euclidean and ix.config.m == 16
    q = O.fill_uniform(100 * d, 8).reshape(100, d)
    for k, ef in ((10, 10), (10, 64), (5, 200)):
        got_ids, got_d, got_n = ix.search_array(q, k, ef)
        rids, rd, rc = h.search(q, k, ef)
        assert np.array_equal(got_n, rc)
        bad = np.nonzero(np.any(got_ids[:, :k].astype(np.int64) != rids * 3 + 11, axis=1))[0]
        assert len(bad) == 0, (k, ef, bad[:5], got_ids[bad[:2]], rids[bad[:2]] * 3 + 11, got_d[bad[:2]], rd[bad[:2]])
        assert np.array_equal(got_d, rd)


def test_dump_of_gpu_built_index_round_trips(tmp_path):
    n, d = 4000, 48
    x = O.fill_uniform(n * d, 21).reshape(n, d)
    ix = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=12, ef_construction=80, ef_search=50))
    ix.add_array(x, np.arange(n, dtype=np.uint64) + 5)
    ix.file_dump(str(tmp_path), "gpu")
    # structure: an independent parse of the dump equals the exported graph
    dump = H.read_dump(str(tmp_path / "gpu"))
    g = ix.export_graph()
    assert dump["nb_point"] == n and dump["dim"] == d and dump["m"] == 12 and dump["ef"] == 80
    assert len(dump["points"]) == n and np.array_equal(dump["vectors"][5 + 17], x[17])
    rows = {(p["layer"], p["rank"]): p["origin"] - 5 for p in dump["points"]}
    for p in dump["points"][::97]:
        row = p["origin"] - 5
        assert p["layer"] == g["levels"][row]
        nb0 = [rows[(lay, r)] for _, lay, r, _ in p["lists"][0]]
        assert nb0 == list(g["col0"][g["row_ptr0"][row]:g["row_ptr0"][row + 1]])
        dists = [dd for *_, dd in p["lists"][0]]
        ref = O.distance_matrix(x[row:row + 1], x[nb0], "l2")[0] if nb0 else []
        assert np.array_equal(np.asarray(dists, np.float32), np.asarray(ref, np.float32))
    assert rows[(dump["entry"][1], dump["entry"][2])] == g["entry"]
    # reload: the same graph up to the row order (rows are grouped by level)
    back = rv.HnswIndex.file_load(str(tmp_path), "gpu", ef_search=50)
    _, bkeys, _ = back.export_rows()
    bg = back.export_graph()
    to_orig = bkeys.astype(np.int64) - 5
    assert to_orig[bg["entry"]] == g["entry"] and bg["max_level"] == g["max_level"]
    assert np.array_equal(np.asarray(bg["levels"])[np.argsort(to_orig)], g["levels"])
    for r in range(n):
        o = to_orig[r]
        a = list(to_orig[bg["col0"][bg["row_ptr0"][r]:bg["row_ptr0"][r + 1]]])
        b = list(g["col0"][g["row_ptr0"][o]:g["row_ptr0"][o + 1]])
        assert a == b, (r, o, a, b)
    for l in range(1, g["max_level"] + 1):
        assert sorted(to_orig[bg["upper_ids"][l - 1]]) == sorted(
            o for o, jj in zip(g["upper_ids"][l - 1], range(len(g["upper_ids"][l - 1])))
            if g["upper_row_ptr"][l - 1][jj + 1] > g["upper_row_ptr"][l - 1][jj])
        for j, r in enumerate(bg["upper_ids"][l - 1]):
            o = to_orig[r]
            rp = bg["upper_row_ptr"][l - 1]
            a = list(to_orig[bg["upper_col"][l - 1][rp[j]:rp[j + 1]]])
            ids = g["upper_ids"][l - 1]
            jj = int(np.searchsorted(ids, o))
            b = [] if jj == len(ids) or ids[jj] != o else \
                list(g["upper_col"][l - 1][g["upper_row_ptr"][l - 1][jj]:g["upper_row_ptr"][l - 1][jj + 1]])
            assert a == b, (l, r, o, a, b)
    q = O.fill_uniform(200 * d, 22).reshape(200, d)
    a = ix.search_array(q, 10, 50)
    b = back.search_array(q, 10, 50)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


def test_file_load_rejects_bad_files(tmp_path):
    (tmp_path / "bad.hnsw.graph").write_bytes(b"\x00" * 64)
    (tmp_path / "bad.hnsw.data").write_bytes(b"\x00" * 64)
    with pytest.raises(rv.RvxError):
        rv.HnswIndex.file_load(str(tmp_path), "bad")
    with pytest.raises(rv.RvxError):
        rv.HnswIndex.file_load(str(tmp_path), "missing")


@pytest.mark.parametrize("layout,page", [(F.RAW, 0), (F.COLD_TIER, 0), (F.COLD_TIER, 1024)])
def test_feature_files_round_trip(tmp_path, layout, page):
    n, d = 70_001, 40
    x = O.fill_uniform(n * d, 31).reshape(n, d)
    buf = rv.Buffer.from_numpy(x)
    path = str(tmp_path / "feat")
    F.store_features(buf, path, n, d, layout, page)
    data = open(path, "rb").read()
    if layout == F.RAW:
        assert data == x.tobytes()
    else:
        dim, rows, block = struct.unpack_from("<QQQ", data, 0)
        assert (dim, rows) == (d, n) and block % (page or 4096) == 0 and block >= 4 * d
        assert data[24 + 3 * block:24 + 3 * block + 4 * d] == x[3].tobytes()
    back = F.load_features(path, layout, d)
    assert np.array_equal(back.download(np.float32, (n, d)), x)
    part = F.load_features(path, layout, d, row0=1234, rows=999)
    assert np.array_equal(part.download(np.float32, (999, d)), x[1234:2233])


def test_feature_file_from_reference_layout(tmp_path):
    """A cold-tier file written exactly as FeatureStorage::create/write_features would."""
    n, d, page = 500, 24, 4096
    x = O.fill_uniform(n * d, 32).reshape(n, d)
    path = tmp_path / "ref.cold"
    with open(path, "wb") as f:
        f.write(struct.pack("<QQQ", d, n, page))
        for r in x:
            f.write(r.tobytes() + b"\0" * (page - 4 * d))
    back = F.load_features(str(path), F.COLD_TIER)
    assert np.array_equal(back.download(np.float32, (n, d)), x)


def test_hnsw_state_serialize_deserialize():
    d = 16
    x = O.fill_uniform(300 * d, 41).reshape(300, d)
    ix = rv.HnswIndex(d, rv.DistanceMetric.Cosine, rv.HnswConfig(m=8, ef_construction=50, ef_search=40))
    ix.add_batch([(f"doc-{i}", x[i]) for i in range(300)])
    assert ix.remove("doc-7")
    blob = ix.serialize()
    st = F.HnswState.decode(blob)
    assert st.metric == "Cosine" and st.dimensions == d and st.next_idx == 300 and len(st.vectors) == 299
    assert ("doc-8", 8) in st.id_to_idx and (8, "doc-8") in st.idx_to_id
    back = rv.HnswIndex.deserialize(blob)
    assert len(back) == 299 and back.config.m == 8 and back.metric == rv.DistanceMetric.Cosine
    r = back.search(x[8], 1)
    assert r[0].id == "doc-8"
    assert back.serialize() == blob  # same live set, same maps
