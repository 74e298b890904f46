"""Node-range-sharded index search across processes (SURVEY.md §8e option 2; VERDICT r2
"missing" 1 and 4): query broadcast from rank 0, per-shard search, all-gather of every
rank's top-k, GPU merge in ShardedHyperbolicHnsw::search order
(crates/ruvector-hyperbolic-hnsw/src/shard.rs:354-373), result shape
(global_id, SearchResult{id: local_id, distance}).

World 2 and 3 share GPU 0 through the host-staged transport (rvx_comm_init_host) behind
the same broadcast / all-gather calls RCCL serves in production
(tests/sharded_search_worker.py): graph search on oracle-built shard graphs, exact
scans and the VectorIndex shards must equal the merge of the per-shard oracle searches
(ids and distances bit-exact, pruned search included: every shard's Fréchet centroid
and tangent coordinates equal the oracle's bits).
Ragged shards include one smaller than k. The RCCL transport itself is the driver's
8-GPU run.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle as O

rv = pytest.importorskip("ruvector_amd")
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def ball_points(n, d, seed, rmax=0.9):
    r = np.random.default_rng(seed)
    v = r.standard_normal((n, d)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    return (v * (rmax * r.random((n, 1)))).astype(np.float32)


def test_single_process_group_is_a_shifted_search():
    """comm None: the sharded entry point is the shard's own search with ids + id_base,
    local ids beside them, and the reference result shape."""
    d = 16
    x = ball_points(800, d, 7)
    h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=2))
    h.insert_batch(x)
    q = ball_points(30, d, 8)
    grp = rv.ShardedHyperbolicSearch(h, None, 1000)
    for mode in ("search", "exact"):
        gid, lid, dist, cnt = grp.search_batch(q, 7, 0, mode)
        ids, dd, c = (h.search_batch(q, 7) if mode == "search" else h.brute_force(q, 7))
        assert np.array_equal(lid, ids) and np.array_equal(gid, np.where(ids >= 0, ids + 1000, -1))
        assert np.array_equal(dist, dd)
    res = grp.search(q[0], 5)
    assert [(g, r.id) for g, r in res] == [(int(i) + 1000, int(i)) for i in h.search_batch(q[:1], 5)[0][0]]
    # the in-process ShardedHyperbolicHnsw returns the same shape
    sh = rv.ShardedHyperbolicHnsw()
    sh.add_shard(x[:300])
    sh.add_shard(x[300:])
    for g, r in sh.search(q[1], 6):
        assert g == r.id + (300 if g >= 300 else 0)


# world 8: the 8-way merge, broadcast and all-gather the driver's 8-GPU
# C5 run takes, with 8 ranks on one GPU — ragged shards, one smaller than k, one empty
@pytest.mark.parametrize("offsets,dim", [([0, 1500, 3001], 32), ([0, 7, 1600, 3000], 32), ([0, 700, 1500], 1024),
                                         ([0, 3, 400, 1000, 1000, 1500, 2100, 2600, 3001], 32)])
def test_sharded_search_multi_rank(offsets, dim, tmp_path):
    world = len(offsets) - 1
    port = _free_port()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    procs = []
    for r in range(world):
        out = tmp_path / f"rank{r}.json"
        procs.append((out, subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "tests", "sharded_search_worker.py"), str(world), str(r), str(port),
             str(out), ",".join(map(str, offsets)), str(dim)], env=env, start_new_session=True)))
    try:
        for _, p in procs:
            p.wait(timeout=150 if world <= 3 else 400)
    finally:
        for _, p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
    res = [json.loads(o.read_text()) for o, _ in procs]
    for r in res:
        assert "error" not in r, r.get("error")
        bad = [k for k, v in r["checks"].items() if not v]
        assert not bad, (r["rank"], bad)
        assert r["pruned_recall_vs_oracle"] >= 0.98, r
