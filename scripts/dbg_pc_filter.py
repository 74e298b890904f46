"""Debug: K10 Poincaré filter vs the VALU scan on C5 points; prints mismatching queries."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ruvector_amd as rv  # noqa: E402


def ball_points(n, d, seed, rmax=0.9):
    r = np.random.default_rng(seed)
    v = r.standard_normal((n, d)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    return (v * (rmax * r.random((n, 1)))).astype(np.float32)


for d, n, wide in [(1024, 70000, "1"), (1024, 70000, "0"), (64, 30000, "1"), (64, 30000, "0"), (768, 70000, "1")]:
    x = ball_points(n, d, 80 + d)
    q = ball_points(300, d, 81 + d)
    h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=1, ef_construction=16, max_connections=4, max_connections_0=8),
                          dim=d)
    h.insert_batch(x)
    os.environ["RVX_SCAN_WIDE"] = wide
    os.environ["RVX_SCAN_MFMA"] = "2"
    ids, dist, _ = h.brute_force(q, 10)
    st = rv.scan_last_stats()
    os.environ["RVX_SCAN_MFMA"] = "0"
    vids, vdist, _ = h.brute_force(q, 10)
    bad = np.where(~np.all(ids == vids, axis=1))[0]
    print(f"d {d} wide {wide}: stats {st}; mismatching queries {len(bad)}", flush=True)
    for qi in bad[:3]:
        print("  q", qi, "mfma", ids[qi].tolist(), dist[qi].tolist())
        print("  q", qi, "valu", vids[qi].tolist(), vdist[qi].tolist())
        missing = set(vids[qi].tolist()) - set(ids[qi].tolist())
        print("  missing rows", sorted(missing), "norms", [float(np.linalg.norm(x[m])) for m in sorted(missing)])
