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


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, script, argv):
    """`--gpus N` without a launcher: run N copies of `script` as ranks 0..N-1 of one job
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, as
    torch.distributed.run would), each a child process of this one — this process has
    not touched the GPU and never execs. Rank 0 writes to this process's stdout (the
    bench's JSON line); the other ranks' stdout goes to stderr. When a rank fails the
    others are stopped (they would wait in a collective) and its status is returned."""
    import signal
    import subprocess
    import sys
    import time
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env,
                                      stdout=None if r == 0 else sys.stderr, start_new_session=True))

    def stop_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except OSError:
                    pass
        t_end = time.monotonic() + 20
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()

    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print(f"[spawn_ranks] rank {r} exited with status {c}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                stop_all()
                return c if c > 0 else 1
            if all(c == 0 for c in codes):
                return 0
            time.sleep(0.2)
    except KeyboardInterrupt:
        stop_all()
        raise
