"""Host-staged librvx communicator over torch.distributed (gloo) — test
infrastructure: lets several ranks share one GPU, which RCCL refuses. The
product ships only the C hook (rvx_comm_init_host) and RCCL (RcclComm)."""
import ctypes as C

from ruvector_amd import _lib as L
from ruvector_amd.shard import HOST_EXCHANGE_FN


class HostComm:
    """librvx communicator over the host-staged transport (rvx_comm_init_host): the
    same per-round row exchange the *_forward_exchange entry points run over RCCL,
    moved through torch.distributed point-to-point sends (gloo). Lets several ranks
    share one GPU (tests) — RCCL refuses two ranks on one device."""

    def __init__(self, world: int, rank: int, group=None):
        import torch.distributed as dist
        self.world, self.rank, self._group = world, rank, group
        self._dist = dist

        def exchange(_user, send, send_bytes, recv, recv_bytes):
            try:
                import torch
                reqs = []
                if send_bytes:
                    st = torch.frombuffer((C.c_char * send_bytes).from_address(send), dtype=torch.uint8)
                    for k in range(1, world):
                        reqs.append(dist.isend(st, (rank + k) % world, group=group))
                for k in range(1, world):
                    p = (rank - k) % world
                    if recv_bytes[p]:
                        rt = torch.frombuffer((C.c_char * recv_bytes[p]).from_address(recv[p]), dtype=torch.uint8)
                        reqs.append(dist.irecv(rt, p, group=group))
                for r in reqs:
                    r.wait()
                return 0
            except Exception:  # a status, never an exception through the C frames
                import traceback
                traceback.print_exc()
                return 1

        self._fn = HOST_EXCHANGE_FN(exchange)  # keep the trampoline alive
        h = C.c_void_p()
        L.call("rvx_comm_init_host", int(world), int(rank), self._fn, None, C.byref(h))
        self._h = h

    def __del__(self):
        try:
            if self._h:
                L.call("rvx_comm_destroy", self._h)
                self._h = None
        except Exception:
            pass
