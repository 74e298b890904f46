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
