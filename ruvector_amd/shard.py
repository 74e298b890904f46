"""Node-range sharding across GPUs of one node.

One process per GPU. Rank r owns destination rows [r*n_local, (r+1)*n_local)
and the CSR rows of those nodes (global column ids). Per GNN layer the only
exchange is an all-gather of the node table (the halo is effectively the
whole graph for HNSW-like topologies); HNSW shards merge per-shard top-k.

The exchange is pluggable so the same driver runs over RCCL on MI355X
(RcclComm, device buffers, librvx) and over torch.distributed gloo in the
tests (tests/host_comm.py, tests/test_shard_gloo.py); the package itself
imports no torch. The product side needs no collective
library of its own: the RCCL id travels over a stdlib TCP rendezvous
(rendezvous_unique_id) and barriers / clock maxima are RCCL all-reduces.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Callable, List, Sequence, Tuple

import numpy as np

from . import _lib as L
from .device import Buffer


@dataclass(frozen=True)
class ShardPlan:
    num_nodes: int
    world: int

    def rows(self, rank: int) -> Tuple[int, int]:
        """[begin, end) of the rows owned by `rank` (contiguous, as even as possible)."""
        base, extra = divmod(self.num_nodes, self.world)
        begin = rank * base + min(rank, extra)
        return begin, begin + base + (1 if rank < extra else 0)

    def owner(self, node: int) -> int:
        base, extra = divmod(self.num_nodes, self.world)
        cut = extra * (base + 1)
        return node // (base + 1) if node < cut else extra + (node - cut) // max(base, 1)

    def equal(self) -> bool:
        return self.num_nodes % self.world == 0


# The host-staged transport (rvx_comm_init_host) takes a C callback
# rvx_host_exchange_fn; tests/host_comm.py implements one over gloo.
HOST_EXCHANGE_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_void_p),
                               C.POINTER(C.c_int64))


PLAN_SAGE, PLAN_WHOLE = 0, 1


def exchange_plan(kind: int, offsets: Sequence[int]) -> List[List[Tuple[int, int]]]:
    """The C++ round plan (rvx_exchange_plan) the *_forward_exchange entry points run:
    rounds[c][p] = (r0, rows) rank p ships in round c."""
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    world = len(off) - 1
    n = C.c_int32(0)
    L.call("rvx_exchange_plan", int(kind), off.ctypes.data_as(C.c_void_p), world, C.byref(n), None, None)
    r0 = np.empty((n.value, world), np.int64)
    rows = np.empty((n.value, world), np.int64)
    L.call("rvx_exchange_plan", int(kind), off.ctypes.data_as(C.c_void_p), world, C.byref(n),
           r0.ctypes.data_as(C.c_void_p), rows.ctypes.data_as(C.c_void_p))
    return [[(int(r0[c, p]), int(rows[c, p])) for p in range(world)] for c in range(n.value)]


def rendezvous_unique_id(rank: int, world: int, make_id: Callable[[], bytes], addr: str = None, port: int = None,
                         timeout: float = 300.0) -> bytes:
    """Hand rank 0's communicator id to every rank over plain TCP (no launcher
    collective library): rank 0 serves `make_id()` on (MASTER_ADDR,
    MASTER_PORT + 17) to each of the world-1 peers, which connect with retry.
    The offset keeps clear of the launcher's own store on MASTER_PORT."""
    import os
    import socket
    import time
    if world <= 1:
        return make_id()
    addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = (port if port is not None else int(os.environ.get("MASTER_PORT", "29500"))) + 17
    if rank == 0:
        uid = make_id()
        with socket.create_server((addr, port), reuse_port=False) as srv:
            srv.settimeout(timeout)
            for _ in range(world - 1):
                conn, _a = srv.accept()
                with conn:
                    conn.sendall(len(uid).to_bytes(4, "little") + uid)
        return uid
    deadline = time.monotonic() + timeout
    while True:
        try:
            with socket.create_connection((addr, port), timeout=10.0) as conn:
                buf = b""
                while len(buf) < 4 or len(buf) < 4 + int.from_bytes(buf[:4], "little"):
                    chunk = conn.recv(4096)
                    if not chunk:
                        raise ConnectionError("rendezvous closed early")
                    buf += chunk
                return buf[4:4 + int.from_bytes(buf[:4], "little")]
        except (ConnectionRefusedError, ConnectionError, socket.timeout, OSError):
            if time.monotonic() > deadline:
                raise
            time.sleep(0.2)


REDUCE_SUM, REDUCE_MAX, REDUCE_MIN = 0, 1, 2


def comm_traffic(comm) -> tuple:
    """(sent, received) payload bytes of a librvx communicator (RcclComm / SocketComm) since it
    was made: every exchange round, broadcast and all-gather (rvx_comm_traffic)."""
    sent, recv = C.c_int64(), C.c_int64()
    L.call("rvx_comm_traffic", comm._h, C.byref(sent), C.byref(recv))
    return sent.value, recv.value


def comm_selfcheck(comm) -> tuple:
    """(rows, mismatched 32-bit words) of the RVX_COMM_SELF_P2P record check: the GraphSAGE
    exchange's compact records after an RCCL round trip to the rank itself, expanded by the
    receivers' unpack kernel and compared with their source rows (rvx_comm_selfcheck)."""
    rows, bad = C.c_int64(), C.c_int64()
    L.call("rvx_comm_selfcheck", comm._h, C.byref(rows), C.byref(bad))
    return rows.value, bad.value


class RcclComm:
    """RCCL communicator of librvx (one per process/GPU)."""

    @classmethod
    def from_env(cls) -> "RcclComm":
        """One communicator over the launcher's RANK / WORLD_SIZE, id by rendezvous_unique_id."""
        import os
        world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
        return cls(world, rank, rendezvous_unique_id(rank, world, cls.unique_id))

    def __init__(self, world: int, rank: int, unique_id: bytes):
        arr = (C.c_uint8 * L.COMM_ID_BYTES).from_buffer_copy(unique_id)
        h = C.c_void_p()
        L.call("rvx_comm_init", arr, int(world), int(rank), C.byref(h))
        self._h, self.world, self.rank = h, world, rank

    @staticmethod
    def unique_id() -> bytes:
        arr = (C.c_uint8 * L.COMM_ID_BYTES)()
        L.call("rvx_comm_unique_id", arr)
        return bytes(arr)

    def allgather(self, send: Buffer, count: int, recv: Buffer) -> None:
        L.call("rvx_comm_allgather_f32", self._h, send.handle, int(count), recv.handle)

    def max(self, value: float) -> float:
        v = C.c_double(value)
        L.call("rvx_comm_allreduce_max_f64", self._h, C.byref(v))
        return v.value

    def allreduce(self, values: Sequence[float], op: int = REDUCE_SUM) -> List[float]:
        arr = (C.c_double * len(values))(*[float(v) for v in values])
        L.call("rvx_comm_allreduce_f64", self._h, arr, len(values), int(op))
        return list(arr)

    def barrier(self) -> None:
        """Every rank's library stream drained and every rank arrived."""
        self.allreduce([0.0])

    def __del__(self):
        try:
            if self._h:
                L.call("rvx_comm_destroy", self._h)
                self._h = None
        except Exception:
            pass


class SocketComm:
    """librvx communicator over the host-staged transport (rvx_comm_init_host) with a
    stdlib TCP full mesh between the ranks: the *_forward_exchange rounds, sharded-search
    broadcasts and all-gathers move through host memory and sockets, and the scalar
    all-reduces (barrier, max-over-ranks clock, sums) go through rank 0. No torch, no
    RCCL: it lets several ranks share one GPU (RCCL refuses two ranks on one device), so
    the multi-rank path runs end to end where only one GPU exists. Same interface as
    RcclComm (_h, allreduce, max, barrier)."""

    PORT_OFFSET = 23  # MASTER_PORT + 23 + rank: clear of the launcher store and the RCCL rendezvous

    @classmethod
    def from_env(cls) -> "SocketComm":
        import os
        return cls(int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
                   os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ.get("MASTER_PORT", "29500")))

    def __init__(self, world: int, rank: int, addr: str = "127.0.0.1", port: int = 29500, timeout: float = 300.0):
        import socket
        import time
        self.world, self.rank = world, rank
        self._peers = {}
        base = port + self.PORT_OFFSET
        srv = socket.create_server((addr, base + rank)) if rank < world - 1 else None
        try:
            # connect to every lower rank (announcing our rank), accept every higher one
            for p in range(rank):
                deadline = time.monotonic() + timeout
                while True:
                    try:
                        s = socket.create_connection((addr, base + p), timeout=10.0)
                        break
                    except OSError:
                        if time.monotonic() > deadline:
                            raise
                        time.sleep(0.1)
                s.sendall(rank.to_bytes(4, "little"))
                self._peers[p] = s
            if srv is not None:
                srv.settimeout(timeout)
                for _ in range(world - 1 - rank):
                    s, _a = srv.accept()
                    p = int.from_bytes(self._recv(s, 4), "little")
                    self._peers[p] = s
        finally:
            if srv is not None:
                srv.close()
        for s in self._peers.values():
            s.settimeout(None)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._fn = HOST_EXCHANGE_FN(self._exchange)  # keep the trampoline alive
        h = C.c_void_p()
        L.call("rvx_comm_init_host", int(world), int(rank), self._fn, None, C.byref(h))
        self._h = h

    @staticmethod
    def _recv(s, n: int, out=None):
        buf = out if out is not None else bytearray(n)
        view = memoryview(buf)
        got = 0
        while got < n:
            k = s.recv_into(view[got:], n - got)
            if k == 0:
                raise ConnectionError("peer closed the connection")
            got += k
        return buf

    def _exchange(self, _user, send, send_bytes, recv, recv_bytes) -> int:
        """rvx_host_exchange_fn: ship send[0:send_bytes) to every peer, fill recv[p] with
        recv_bytes[p] from peer p. Frames carry their length; sends run on threads so no
        pair of ranks waits on each other's full socket buffers."""
        import threading
        try:
            errs = []
            payload = (C.c_char * send_bytes).from_address(send) if send_bytes else None

            def ship(s):
                try:
                    s.sendall(int(send_bytes).to_bytes(8, "little"))
                    s.sendall(memoryview(payload).cast("B"))
                except Exception as e:  # noqa: BLE001
                    errs.append(e)

            ts = [threading.Thread(target=ship, args=(s,)) for p, s in sorted(self._peers.items())] if send_bytes else []
            for t in ts:
                t.start()
            for p, s in sorted(self._peers.items()):
                nb = int(recv_bytes[p])
                if nb == 0:
                    continue
                hdr = int.from_bytes(self._recv(s, 8), "little")
                if hdr != nb:
                    raise ValueError(f"rank {self.rank}: expected {nb} bytes from rank {p}, got a frame of {hdr}")
                dst = (C.c_char * nb).from_address(recv[p])
                self._recv(s, nb, memoryview(dst).cast("B"))
            for t in ts:
                t.join()
            if errs:
                raise errs[0]
            return 0
        except Exception:  # a status, never an exception through the C frames
            import traceback
            traceback.print_exc()
            return 1

    def allreduce(self, values: Sequence[float], op: int = REDUCE_SUM) -> List[float]:
        """Element-wise sum / max / min of float64 values over the ranks (through rank 0)."""
        import struct
        vals = [float(v) for v in values]
        n = len(vals)
        fmt = f"<{n}d"
        if self.rank == 0:
            acc = list(vals)
            for p in sorted(self._peers):
                got = struct.unpack(fmt, bytes(self._recv(self._peers[p], 8 * n)))
                for i, v in enumerate(got):
                    acc[i] = acc[i] + v if op == REDUCE_SUM else max(acc[i], v) if op == REDUCE_MAX else min(acc[i], v)
            out = struct.pack(fmt, *acc)
            for p in sorted(self._peers):
                self._peers[p].sendall(out)
            return acc
        s = self._peers[0]
        s.sendall(struct.pack(fmt, *vals))
        return list(struct.unpack(fmt, bytes(self._recv(s, 8 * n))))

    def max(self, value: float) -> float:
        return self.allreduce([value], REDUCE_MAX)[0]

    def barrier(self) -> None:
        """Every rank's library stream drained and every rank arrived."""
        L.call("rvx_synchronize")
        self.allreduce([0.0])

    def close(self) -> None:
        try:
            if getattr(self, "_h", None):
                L.call("rvx_comm_destroy", self._h)
                self._h = None
        finally:
            for s in self._peers.values():
                s.close()
            self._peers = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_from_env(transport: str = "rccl"):
    """The communicator of a launched rank (None at world 1): RCCL over xGMI, or the
    stdlib-socket host transport (`transport="host"`, several ranks per GPU)."""
    import os
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    return SocketComm.from_env() if transport == "host" else RcclComm.from_env()


PIPE_CHUNKS = 48         # RVX_SAGE_CHUNKS default (api_graph.cpp sage_chunks_for)
PIPE_MIN_ROWS = 16384    # rows per chunk below which a layer is not chunked


def chunk_count(n_rows: int, chunks: int = PIPE_CHUNKS) -> int:
    """Row chunks of one layer pipeline (mirror of sage_chunks_for)."""
    return chunks if n_rows >= chunks * PIPE_MIN_ROWS else 1


def chunk_step(n_rows: int, chunks: int) -> int:
    """Rows per chunk, a multiple of the GEMM's 128-row tile (mirror of chunk_step)."""
    return (-(-n_rows // chunks) + 127) // 128 * 128


def exchange_rounds(offsets: Sequence[int]) -> List[List[Tuple[int, int]]]:
    """The p2p rounds of rvx_sage_forward_exchange: every rank uses the chunk
    count of the largest shard, and in round c rank p ships its rows
    [r0, r0+rows) (possibly empty) to every peer. Returns rounds[c][p]."""
    world = len(offsets) - 1
    sizes = [offsets[p + 1] - offsets[p] for p in range(world)]
    chunks = chunk_count(max(sizes))
    rounds = []
    for c in range(chunks):
        rr = []
        for p in range(world):
            st = chunk_step(sizes[p], chunks)
            b = min(sizes[p], c * st)
            rr.append((offsets[p] + b, min(st, sizes[p] - b)))
        rounds.append(rr)
    return rounds


def merge_topk(parts: Sequence[Tuple[np.ndarray, np.ndarray]], k: int) -> Tuple[np.ndarray, np.ndarray]:
    """ShardedHyperbolicHnsw::search merge (crates/ruvector-hyperbolic-hnsw/src/shard.rs:354-373):
    concatenate per-shard (global id, distance) lists, sort by distance (ties by id), truncate k."""
    ids = np.concatenate([p[0] for p in parts], axis=1)
    d = np.concatenate([p[1] for p in parts], axis=1)
    out_i = np.empty((ids.shape[0], k), ids.dtype)
    out_d = np.empty((ids.shape[0], k), d.dtype)
    for q in range(ids.shape[0]):
        order = np.lexsort((ids[q], d[q]))[:k]
        out_i[q], out_d[q] = ids[q][order], d[q][order]
    return out_i, out_d


def sharded_layers(x_local, layers: Sequence, plan: ShardPlan, rank: int,
                   allgather: Callable, forward_rows: Callable):
    """Run `layers` over a node-range-sharded graph.

    allgather(local) -> full table; forward_rows(layer, full_table, row_begin, row_end) -> owned rows.
    Returns this rank's rows of the last layer's output.
    """
    h = x_local
    b, e = plan.rows(rank)
    for layer in layers:
        full = allgather(h)
        h = forward_rows(layer, full, b, e)
    return h
