"""Multi-process (world_size 2, gloo on CPU) test of the node-range sharding
driver (ruvector_amd/shard.py): per-layer all-gather of the node table + each
rank transforming its own rows must reproduce the single-process forward;
per-shard top-k merged must equal the global top-k.

The per-rank compute here is the oracle (test double for the HIP layer); the
exchange is torch.distributed.all_gather over gloo — the same driver runs over
RCCL with HBM buffers in bench.py.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import oracle as O
    from ruvector_amd.shard import ShardPlan, merge_topk, sharded_layers

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, d, deg = 203, 16, 5  # ragged: 203 rows over 2 ranks
        plan = ShardPlan(n, world)
        x = O.fill_uniform(n * d, 1).reshape(n, d)
        rp, col = O.random_csr(n, deg, 2)
        wn, ws = O.sage_init(d, d, 0), O.sage_init(d, d, 1000)
        b, e = plan.rows(rank)

        def allgather(local):
            sizes = [plan.rows(r)[1] - plan.rows(r)[0] for r in range(world)]
            bufs = [torch.zeros((s, d), dtype=torch.float32) for s in sizes]
            t = torch.from_numpy(np.ascontiguousarray(local))
            # gloo all_gather needs equal sizes: pad to the max
            m = max(sizes)
            pad = torch.zeros((m, d), dtype=torch.float32)
            pad[:t.shape[0]] = t
            outs = [torch.zeros((m, d), dtype=torch.float32) for _ in range(world)]
            dist.all_gather(outs, pad)
            return np.concatenate([o[:s].numpy() for o, s in zip(outs, sizes)])

        def forward_rows(layer, full, rb, re):
            return O.sage_forward(full, rp, col, wn, ws, rows=(rb, re - rb))

        mine = sharded_layers(x[b:e], [0, 1], plan, rank, allgather, forward_rows)
        ref = O.sage_forward(O.sage_forward(x, rp, col, wn, ws), rp, col, wn, ws)[b:e]
        ok_gnn = bool(np.array_equal(mine, ref))

        # HNSW/flat shard merge: each rank owns a row range of the corpus
        base = O.fill_uniform(500 * 8, 3).reshape(500, 8)
        qv = O.fill_uniform(12 * 8, 4).reshape(12, 8)
        p2 = ShardPlan(500, world)
        sb, se = p2.rows(rank)
        li, ld = O.flat_search(base[sb:se], qv, 7, "l2")
        li = li + sb
        gi = [torch.zeros((12, 7), dtype=torch.int64) for _ in range(world)]
        gd = [torch.zeros((12, 7), dtype=torch.float32) for _ in range(world)]
        dist.all_gather(gi, torch.from_numpy(li))
        dist.all_gather(gd, torch.from_numpy(ld))
        mi, md = merge_topk([(a.numpy(), b_.numpy()) for a, b_ in zip(gi, gd)], 7)
        fi, fd = O.flat_search(base, qv, 7, "l2")
        ok_merge = bool(np.array_equal(mi, fi) and np.array_equal(md, fd))
        q.put((rank, ok_gnn, ok_merge))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_node_range_shards_match_single_process(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert res == [(r, True, True) for r in range(world)]


def _exchange_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from ruvector_amd.shard import exchange_rounds

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # ragged shards, one far below the pipelining threshold
        # the largest shard above PIPE_CHUNKS * PIPE_MIN_ROWS; at world 8 also an empty shard and a
        # one-row shard (they send empty blocks in most rounds)
        sizes = ([900_000, 150_001, 5_000] if world <= 3 else
                 [900_000, 150_001, 5_000, 0, 70_000, 1, 300_000, 20_000])[:world]
        offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        n, d = int(offsets[-1]), 3
        full = np.arange(n * d, dtype=np.float32).reshape(n, d)
        table = np.zeros_like(full)
        b, e = offsets[rank], offsets[rank + 1]
        rounds = exchange_rounds(offsets)
        mine = []
        for rr in rounds:
            r0, rows = rr[rank]
            mine.append((r0, rows))
            table[r0:r0 + rows] = full[r0:r0 + rows]  # "compute" of this chunk
            reqs = []
            for k in range(1, world):  # same rotated peer order as comm_exchange_rows
                p = (rank + k) % world
                if rows > 0:
                    reqs.append(dist.isend(torch.from_numpy(table[r0:r0 + rows].copy()), p))
                pr0, prows = rr[p]
                if prows > 0:
                    buf = torch.zeros((prows, d), dtype=torch.float32)
                    reqs.append((dist.irecv(buf, p), pr0, buf))
            for r in reqs:
                if isinstance(r, tuple):
                    r[0].wait()
                    table[r[1]:r[1] + r[2].shape[0]] = r[2].numpy()
                else:
                    r.wait()
        covered = sum(rows for _, rows in mine) == e - b and mine[0][0] == b and all(
            mine[i][0] + mine[i][1] == mine[i + 1][0] for i in range(len(mine) - 1) if mine[i + 1][1] > 0)
        q.put((rank, bool(np.array_equal(table, full)), bool(covered), len(rounds)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_chunked_halo_exchange_protocol(world):
    """rvx_sage_forward_exchange's round plan (mirrored by shard.exchange_rounds)
    reconstructs the full table on every rank with ragged shards."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    res = sorted(q.get(timeout=5) for _ in range(world))
    from ruvector_amd.shard import PIPE_CHUNKS
    assert res == [(r, True, True, PIPE_CHUNKS) for r in range(world)]


def test_shard_plan_rows_cover_and_owner():
    sys.path.insert(0, ROOT)
    from ruvector_amd.shard import ShardPlan
    for n, w in ((10, 3), (8, 8), (1000003, 8), (5, 8)):
        p = ShardPlan(n, w)
        spans = [p.rows(r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
        for node in range(0, n, max(1, n // 97)):
            r = p.owner(node)
            assert spans[r][0] <= node < spans[r][1]


# ---- the C++ round plan and the host-staged transport (no GPU needed) --------
@pytest.mark.parametrize("offsets", [[0, 1000], [0, 500, 1001], [0, 60000, 100000, 150001],
                                     [0, 400000, 800000], [0, 393216 * 2, 393216 * 2 + 5, 393216 * 3],
                                     [0, 9000, 30000, 30000, 66000, 80000, 101000, 120000, 150001],
                                     [1250000 * p for p in range(9)]])
def test_exchange_plan_matches_mirror(offsets):
    """rvx_exchange_plan (the plan rvx_sage_forward_exchange runs, api_graph.cpp
    exchange_plan) equals the Python mirror shard.exchange_rounds; the whole-shard
    plan of the RuvectorLayer / attention exchange is one round of full shards."""
    from ruvector_amd import shard
    assert shard.exchange_plan(shard.PLAN_SAGE, offsets) == shard.exchange_rounds(offsets)
    whole = shard.exchange_plan(shard.PLAN_WHOLE, offsets)
    assert whole == [[(offsets[p], offsets[p + 1] - offsets[p]) for p in range(len(offsets) - 1)]]
    # every rank's rows are covered exactly once across the rounds
    for p in range(len(offsets) - 1):
        got = [r for rnd in shard.exchange_plan(shard.PLAN_SAGE, offsets) for r in [rnd[p]] if r[1]]
        covered = np.concatenate([np.arange(a, a + n) for a, n in got]) if got else np.zeros(0, np.int64)
        assert np.array_equal(covered, np.arange(offsets[p], offsets[p + 1]))


def _host_comm_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import ctypes as C
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from host_comm import HostComm

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = HostComm(world, rank)
        sizes = [3 + 2 * p if p != 1 else 0 for p in range(world)]  # rank 1 sends nothing
        send = np.full(max(sizes[rank], 1), 10.0 * rank + 1, np.float32)
        recv = [np.zeros(max(sizes[p], 1), np.float32) for p in range(world)]
        ptrs = (C.c_void_p * world)(*[None if p == rank else recv[p].ctypes.data for p in range(world)])
        nbytes = (C.c_int64 * world)(*[0 if p == rank else sizes[p] * 4 for p in range(world)])
        rc = comm._fn(None, send.ctypes.data, sizes[rank] * 4, ptrs, nbytes)
        ok = rc == 0 and all(np.all(recv[p][:sizes[p]] == 10.0 * p + 1) for p in range(world) if p != rank)
        # broadcast shape (comm_broadcast_bytes): only the root (rank world-1) sends,
        # every other rank receives from the root alone
        root = world - 1
        blk = np.arange(7, dtype=np.float32) + 100.0
        got = np.zeros(7, np.float32)
        ptrs = (C.c_void_p * world)(*[got.ctypes.data if (p == root and rank != root) else None for p in range(world)])
        nbytes = (C.c_int64 * world)(*[28 if (p == root and rank != root) else 0 for p in range(world)])
        rc = comm._fn(None, blk.ctypes.data, 28 if rank == root else 0, ptrs, nbytes)
        ok = ok and rc == 0 and (rank == root or np.array_equal(got, blk))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_host_transport_moves_every_block(world):
    """HostComm's exchange callback (the host-staged transport behind rvx_comm_init_host)
    delivers each rank's block to every peer, ragged and empty blocks included."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_host_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res


def _rdv_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    from ruvector_amd.shard import rendezvous_unique_id
    made = []

    def make():
        made.append(1)
        return bytes(range(128))[::-1] + b"rank0"

    uid = rendezvous_unique_id(rank, world, make, addr="127.0.0.1", port=port, timeout=60.0)
    q.put((rank, uid, len(made)))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tcp_rendezvous_hands_rank0_id_to_every_rank(world):
    """bench.py's multi-GPU bootstrap without torch.distributed: rank 0's RCCL id
    (here a stand-in byte string) reaches every rank over the stdlib TCP
    rendezvous; only rank 0 makes an id."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rdv_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
    ids = {uid for _, uid, _ in got}
    assert len(ids) == 1 and next(iter(ids)).endswith(b"rank0")
    assert sorted(m for _, _, m in got) == [0] * (world - 1) + [1]
