#!/usr/bin/env python3
"""K10 in-kernel clock (MI355X_MICROARCH.md DVFS item 6): run the exact-scan
filter at 10M x 768 / 10k queries back to back for >= `--seconds` on a diagnostic build
(variants/librvx_scanclk.so: k_scan.hip with -DRVX_SCAN_CLOCK, which stamps s_memtime and
s_memrealtime per block and prints the median clock per launch to stderr), so the clock is read
after the chip has settled under the load. Results are identical to the real build; only the
diagnostic build stamps.
usage: RVX_LIB=variants/librvx_scanclk.so python scripts/exp/scan_clock.py [--seconds 6]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--nq", type=int, default=10_000)
    p.add_argument("--seconds", type=float, default=6.0)
    a = p.parse_args()
    import ruvector_amd as rv
    xb = rv.Buffer(a.n * a.d * 4)
    xb.fill_normal(a.n * a.d, 3)
    qb = rv.Buffer(a.nq * a.d * 4)
    qb.fill_normal(a.nq * a.d, 6)
    idx = rv.FlatIndex(a.d, rv.DistanceMetric.Euclidean)
    idx.add_device(xb, a.n, 0)
    ids, dist = rv.Buffer(a.nq * 10 * 8), rv.Buffer(a.nq * 10 * 4)
    t0 = time.perf_counter()
    calls = 0
    while time.perf_counter() - t0 < a.seconds or calls < 3:
        prof = rv.Profiler()
        with prof:
            idx.brute_force_device(qb, a.nq, 10, ids, dist)
            rv.synchronize()
        f_ms, _ = prof.query("scan_filter")
        print(f"call {calls}: scan_filter {f_ms:.2f} ms, {2.0 * a.nq * a.n * a.d / (f_ms * 1e-3) / 1e12:.1f} TFLOP/s f16",
              flush=True)
        calls += 1


if __name__ == "__main__":
    main()
