"""RCCL communicator code run on hardware at world 1.

The multi-rank paths are tested through the host-staged transport (several ranks on one
GPU: RCCL refuses two ranks on one device); this file runs the RCCL side itself on the
one GPU a test box has. `RcclComm` is built through `rendezvous_unique_id` exactly as
`comm_from_env` builds it, and with RVX_COMM_SELF_P2P=1 a one-rank communicator runs every
collective instead of skipping it (api_comm.cpp comm_self_p2p):

  * ncclAllReduce (sum / max / min) and the barrier built on it;
  * ncclAllGather of f32 rows (rvx_comm_allgather_f32);
  * the grouped ncclSend/ncclRecv round of comm_exchange_rows, to the rank itself, inside
    the GraphSAGE (chunked rounds, deferred normalisation), RuvectorLayer and attention
    exchange drivers: outputs bit-identical to the one-process forward;
  * ncclBroadcast + ncclAllGather of the sharded index / hyperbolic searches: results equal
    to the unsharded search;
  * `bench.py --gpus 1 --transport rccl --force-comm`: the RCCL barriers and the
    max-over-ranks clock wrap a real timed step.

Reference pattern: crates/ruvector-hyperbolic-hnsw/src/shard.rs:354-373 (merge of shard
results), SURVEY.md §8e (halo exchange after each layer).
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
import ruvector_amd as rv
from ruvector_amd.shard import REDUCE_MAX, REDUCE_MIN, REDUCE_SUM, RcclComm, rendezvous_unique_id

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def comm():
    c = RcclComm(1, 0, rendezvous_unique_id(0, 1, RcclComm.unique_id))
    yield c
    del c


@pytest.fixture
def self_p2p(monkeypatch):
    monkeypatch.setenv("RVX_COMM_SELF_P2P", "1")


def test_allreduce_barrier_allgather(comm, self_p2p):
    vals = [1.5, -2.25, 3e30, -0.0]
    assert comm.allreduce(vals, REDUCE_SUM) == vals
    assert comm.allreduce(vals, REDUCE_MAX) == vals
    assert comm.allreduce(vals, REDUCE_MIN) == vals
    assert comm.max(7.125) == 7.125
    comm.barrier()
    a = O.fill_uniform(100003, 5)
    send, recv = rv.Buffer.from_numpy(a), rv.Buffer(a.nbytes)
    comm.allgather(send, a.size, recv)
    rv.synchronize()
    assert np.array_equal(recv.download(np.float32, a.shape).view(np.uint32), a.view(np.uint32))


def _sage_pair(comm, layer, g, xb, N, d, off_p, one_p, fn, extra_in, extra_out):
    call = rv._lib.call
    got, ref = rv.Buffer(N * d * 4), rv.Buffer(N * d * 4)
    got.upload(np.full((N, d), np.nan, np.float32))
    call(fn, layer._h, g.handle, xb.handle, *extra_in, got.handle, *extra_out, off_p, comm._h, 1)
    call(fn, layer._h, g.handle, xb.handle, *extra_in, ref.handle, *extra_out, one_p, None, 0)
    rv.synchronize()
    return got.download(np.float32, (N, d)), ref.download(np.float32, (N, d))


def test_sage_exchange_self_p2p_bits(comm, self_p2p, monkeypatch):
    monkeypatch.setenv("RVX_SAGE_CHUNKS", "3")  # three exchange rounds at this size
    N, d, deg = 3 * 16384 + 77, 64, 6
    x = O.fill_uniform(N * d, 91).reshape(N, d)
    rp, col = O.random_csr(N, deg, 92)
    g = rv.Graph.from_csr(rp, col)
    layer = rv.GraphSAGELayer(d, d, num_samples=deg)
    xb = rv.Buffer.from_numpy(x)
    off = np.array([0, N], np.int64)
    off_p = off.ctypes.data_as(C.POINTER(C.c_int64))
    prof = rv.Profiler()
    with prof:
        a, b = _sage_pair(comm, layer, g, xb, N, d, off_p, off_p, "rvx_sage_forward_exchange", (), ())
    assert prof.query("halo_exchange")[1] == 3  # the rounds really ran (through RCCL)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    # deferred normalisation: the 1/|y| column travels in its own round
    iv_a, iv_b = rv.Buffer(N * 4), rv.Buffer(N * 4)
    call = rv._lib.call
    ya, yb = rv.Buffer(N * d * 4), rv.Buffer(N * d * 4)
    call("rvx_sage_forward_exchange2", layer._h, g.handle, xb.handle, None, ya.handle, iv_a.handle, off_p, comm._h, 1)
    call("rvx_sage_forward_exchange2", layer._h, g.handle, xb.handle, None, yb.handle, iv_b.handle, off_p, None, 0)
    rv.synchronize()
    assert np.array_equal(ya.download(np.float32, (N, d)).view(np.uint32), yb.download(np.float32, (N, d)).view(np.uint32))
    assert np.array_equal(iv_a.download(np.float32, (N,)).view(np.uint32), iv_b.download(np.float32, (N,)).view(np.uint32))
    ref = O.sage_forward(x, rp, col, O.sage_init(d, d, 0), O.sage_init(d, d, 1000), rows=(0, 400))
    assert float(np.max(np.abs(a[:400] - ref)) / np.max(np.abs(ref))) <= 1e-5


@pytest.mark.parametrize("row_bytes", [None, "900"])
def test_sage_records_unpacked_behind_rccl(comm, self_p2p, monkeypatch, row_bytes):
    """at world 1 the receive side of the compact records (rows_xchg_unpack)
    never ran behind RCCL. With RVX_COMM_SELF_P2P the rank's own records go out and come back
    through RCCL's p2p path and are expanded by the receivers' unpack kernel into a shadow that
    is compared word for word with the rows they encode (rvx_comm_selfcheck): every row checked,
    no word different — by default and with a budget most rows overflow (those stay dense)."""
    from ruvector_amd.shard import comm_selfcheck
    monkeypatch.setenv("RVX_SAGE_CHUNKS", "3")
    if row_bytes:
        monkeypatch.setenv("RVX_XCHG_ROW_BYTES", row_bytes)
    N, d, deg = 3 * 16384 + 77, 768, 6
    x = O.fill_uniform(N * d, 191).reshape(N, d) - 0.5
    rp, col = O.random_csr(N, deg, 192)
    g = rv.Graph.from_csr(rp, col)
    layer = rv.GraphSAGELayer(d, d, num_samples=deg)
    xb = rv.Buffer.from_numpy(x)
    off = np.array([0, N], np.int64)
    off_p = off.ctypes.data_as(C.POINTER(C.c_int64))
    iv = rv.Buffer(N * 4)
    rows0, bad0 = comm_selfcheck(comm)
    a, b = _sage_pair(comm, layer, g, xb, N, d, off_p, off_p, "rvx_sage_forward_exchange3", (None, None),
                      (iv.handle, None))
    rows1, bad1 = comm_selfcheck(comm)
    assert rows1 - rows0 == N and bad1 == bad0 == 0, (rows0, rows1, bad0, bad1)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert 0.3 < float((a == 0).mean()) < 0.7  # ReLU-sparse rows: the records are the compact form


def test_gnn_and_attention_exchange_self_p2p_bits(comm, self_p2p, monkeypatch):
    from ruvector_amd.attention import EdgeFeaturedAttention, EdgeFeaturedConfig
    monkeypatch.setenv("RVX_SAGE_CHUNKS", "3")
    n, H, heads, deg = 3 * 16384 + 5, 64, 4, 5
    x = O.fill_uniform(n * H, 93).reshape(n, H)
    rp, col = O.random_csr(n, deg, 94)
    ew = O.fill_uniform(len(col), 95, 0.0, 1.0)
    g = rv.Graph.from_csr(rp, col, ew)
    off = np.array([0, n], np.int64)
    rl = rv.RuvectorLayer(H, H, heads, 0.0, seed=7)
    xb = rv.Buffer.from_numpy(x)
    ys, yr = rv.Buffer(n * H * 4), rv.Buffer(n * H * 4)
    rl.forward_exchange(g, xb, ys, off, comm)
    rl.forward_graph_device(xb, g, yr)
    rv.synchronize()
    assert np.array_equal(ys.download(np.float32, (n, H)).view(np.uint32), yr.download(np.float32, (n, H)).view(np.uint32))
    att = EdgeFeaturedAttention(EdgeFeaturedConfig(node_dim=H, edge_dim=1, num_heads=heads))
    eb = rv.Buffer.from_numpy(ew)
    zs, zr = rv.Buffer(n * H * 4), rv.Buffer(n * H * 4)
    att.forward_exchange(g, yr, eb, zs, off, comm)
    att.forward_graph_device(yr, g, eb, zr)
    rv.synchronize()
    assert np.array_equal(zs.download(np.float32, (n, H)).view(np.uint32), zr.download(np.float32, (n, H)).view(np.uint32))


def test_sharded_searches_self_p2p(comm, self_p2p):
    n, d, nq, k = 20000, 64, 300, 10
    x = O.fill_uniform(n * d, 96).reshape(n, d)
    q = O.fill_uniform(nq * d, 97).reshape(nq, d)
    idx = rv.FlatIndex(d, rv.DistanceMetric.Euclidean)
    idx.add_array(x, np.arange(n, dtype=np.uint64))
    ids, dist, cnt = idx.sharded_search_array(comm, q, k, exact=True)
    rids, rd = O.flat_search(x, q, k, "l2")
    assert np.array_equal(ids.astype(np.int64), rids) and np.array_equal(dist, rd)
    assert np.all(cnt == k)
    # hyperbolic: broadcast + all-gather + merge on the GPU, exact mode
    from ruvector_amd.hyperbolic import HyperbolicHnsw, HyperbolicHnswConfig, ShardedHyperbolicSearch
    pts = (O.fill_uniform(4000 * 32, 98).reshape(4000, 32) - 0.5) * 0.05
    h = HyperbolicHnsw(HyperbolicHnswConfig(), dim=32)
    h.insert_batch(pts)
    s = ShardedHyperbolicSearch(h, comm)
    qq = (O.fill_uniform(40 * 32, 99).reshape(40, 32) - 0.5) * 0.05
    gid, _, gd, cnt = s.search_batch(qq, 10, mode="exact")
    bi, bd, _ = h.brute_force(qq, 10)
    assert np.array_equal(np.asarray(gid, np.int64), np.asarray(bi, np.int64))
    assert np.array_equal(np.asarray(gd, np.float32), np.asarray(bd, np.float32)) and np.all(cnt == 10)


def test_bench_force_comm_rccl(tmp_path):
    """bench.py at one GPU with its RCCL communicator forced on: the barrier and the
    max-over-ranks clock are RCCL all-reduces around a real timed step."""
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
                        "--nodes", "200000", "--no-cpu", "--no-scan", "--no-c4", "--no-hnsw", "--no-c5",
                        "--transport", "rccl", "--force-comm", "--check-rows", "512"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["comm"]["transport"] == "rccl" and line["comm"]["forced"] is True
    assert line["comm"]["self_p2p_rounds"] > 0
    # the compact records of every round came back through RCCL and unpacked bit for bit
    chk = line["comm"]["record_selfcheck"]
    assert chk["rows"] > 0 and chk["mismatched_words"] == 0, chk
