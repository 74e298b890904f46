"""Standalone gather-aggregate bandwidth vs node-table size (d=768, deg=32,
mean): separates the per-launch HBM rate from table-size effects (address
translation reach). Usage: python scripts/exp/exp_gather.py [n ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ruvector_amd as rv  # noqa: E402

d, deg = 768, 32
sizes = [int(a) for a in sys.argv[1:]] or [1_000_000, 3_000_000, 10_000_000]
for n in sizes:
    x = rv.Buffer(n * d * 4)
    x.fill_normal(n * d, 3)
    out = rv.Buffer(n * d * 4)
    g = rv.Graph.random(n, deg, 4)
    rv.aggregate(x, g, d, "mean", out)
    rv.synchronize()
    prof = rv.Profiler()
    with prof:
        for _ in range(3):
            rv.aggregate(x, g, d, "mean", out)
        rv.synchronize()
    ms, launches = prof.query("aggregate")
    per = ms / launches
    gb = (n * deg * (4 * d + 4) + n * (8 + 4 * d)) / 1e9
    print(f"n={n} table={n * d * 4 / 1e9:.1f} GB: {per:.2f} ms/launch, {gb / per:.0f} GB/s algorithmic "
          f"(deep={os.environ.get('RVX_AGG_STANDALONE_DEEP', '0')})", flush=True)
    del x, out, g
