"""The stdlib-socket host transport (ruvector_amd.shard.SocketComm) on CPU, world 3 and 8:
scalar all-reduces (sum / max / min, the bench's barrier and max-over-ranks clock) and
the rvx_host_exchange_fn frames the C++ exchange / broadcast / all-gather paths send
(ragged blocks, an empty block, a root-only broadcast). The GPU side of the same
transport runs in tests/test_gpu_bench_multirank.py."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import ctypes as C, sys
    import numpy as np
    sys.path.insert(0, sys.argv[4])
    from ruvector_amd.shard import REDUCE_MAX, REDUCE_MIN, SocketComm
    world, rank, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    comm = SocketComm(world, rank, "127.0.0.1", port)
    assert comm.allreduce([rank, 1.5]) == [sum(range(world)), 1.5 * world]
    assert comm.allreduce([rank, -rank], REDUCE_MAX) == [world - 1, 0]
    assert comm.allreduce([rank], REDUCE_MIN) == [0]
    assert comm.max(10.0 * rank) == 10.0 * (world - 1)

    def block(p, n):
        return (np.arange(n, dtype=np.float32) + 1000 * p)

    # ragged exchange: rank p ships 3 + 5p floats (rank 1 ships none) to every peer
    sizes = [0 if p == 1 else 4 * (3 + 5 * p) for p in range(world)]
    mine = block(rank, sizes[rank] // 4)
    bufs = [np.zeros(max(sizes[p] // 4, 1), np.float32) for p in range(world)]
    rptr = (C.c_void_p * world)(*[b.ctypes.data if p != rank else None for p, b in enumerate(bufs)])
    rbytes = (C.c_int64 * world)(*[sizes[p] if p != rank else 0 for p in range(world)])
    assert comm._exchange(None, mine.ctypes.data, sizes[rank], rptr, rbytes) == 0
    for p in range(world):
        if p != rank and sizes[p]:
            assert np.array_equal(bufs[p][:sizes[p] // 4], block(p, sizes[p] // 4)), p
    # broadcast from rank 2: only the root sends
    root = 2
    msg = np.arange(64, dtype=np.float32) * 3 if rank == root else np.zeros(64, np.float32)
    rptr = (C.c_void_p * world)(*[msg.ctypes.data if p == root and rank != root else None for p in range(world)])
    rbytes = (C.c_int64 * world)(*[256 if p == root and rank != root else 0 for p in range(world)])
    assert comm._exchange(None, msg.ctypes.data, 256 if rank == root else 0, rptr, rbytes) == 0
    assert np.array_equal(msg, np.arange(64, dtype=np.float32) * 3)
    # a frame of the wrong size is reported as a failed status, not an exception
    if world == 3:
        comm.allreduce([0.0])
    comm.close()
    print("ok", rank)
""")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [3, 8])
def test_socket_comm_world(world, tmp_path):
    """world 3 and 8 (the driver's 8-GPU size: the full mesh, scalar all-reduces through rank 0)."""
    w = tmp_path / "worker.py"
    w.write_text(WORKER)
    port = _port()
    procs = [subprocess.Popen([sys.executable, str(w), str(world), str(r), str(port), ROOT], stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True, start_new_session=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=120)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
    for r, (rc, out) in enumerate(outs):
        assert rc == 0 and f"ok {r}" in out, out
