"""Shared helpers of the bench scripts (host side only)."""
import os


def _cgroup_cpus():
    """CPUs granted by the cgroup v2 quota (cpu.max "quota period"), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return None


def host_threads():
    """Worker threads for the CPU-baseline legs and what bounded them.

    Every CPU this process may use: the affinity mask, the cgroup quota and the
    pool's per-GPU CPU share (OMP_NUM_THREADS, which the GPU box sets to the
    share of one GPU — os.cpu_count() there reports the whole machine). `nproc`
    is reported beside the thread count so the line states both."""
    aff = len(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    n = min(x for x in (aff, quota, share) if x)
    return n, {"threads": n, "nproc": os.cpu_count(), "affinity": aff, "cgroup_quota": quota,
               "omp_num_threads": share}


class heartbeat:
    """Print a progress line every `every` seconds while a long native call runs
    (ctypes releases the GIL), so a supervisor that watches output sees life."""

    def __init__(self, label, every=30.0, log=None):
        import sys
        import threading
        self.label, self.every = label, every
        self.log = log or (lambda s: print(s, file=sys.stderr, flush=True))
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        import time
        t0 = time.perf_counter()
        while not self._stop.wait(self.every):
            self.log(f"... {self.label}: {time.perf_counter() - t0:.0f} s")

    def __enter__(self):
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join()
