"""A/B (round 4): K10 wide filter tile on v_mfma_f32_32x32x16_f16 (RVX_SCAN_M16=0) vs
v_mfma_f32_16x16x32_f16 (RVX_SCAN_M16=1), interleaved, one process, same table and
queries (10M x 768 N(0,1) seed 5, 10k queries seed 6, k 10, L2 unless --metric).
Checks that both forms return identical ids and distances."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import ruvector_amd as rv  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=10_000_000)
p.add_argument("--d", type=int, default=768)
p.add_argument("--nq", type=int, default=10_000)
p.add_argument("--reps", type=int, default=3)
p.add_argument("--metric", default="l2")
a = p.parse_args()
metric = {"l2": rv.DistanceMetric.Euclidean, "cosine": rv.DistanceMetric.Cosine, "dot": rv.DistanceMetric.DotProduct}[a.metric]
xb = rv.Buffer(a.n * a.d * 4)
xb.fill_normal(a.n * a.d, 5)
qb = rv.Buffer(a.nq * a.d * 4)
qb.fill_normal(a.nq * a.d, 6)
idx = rv.FlatIndex(a.d, metric)
idx.add_device(xb, a.n, 0)
k = 10
ids_b, dist_b = rv.Buffer(a.nq * k * 8), rv.Buffer(a.nq * k * 4)
os.environ["RVX_SCAN_MFMA"] = "1"
res, out = {}, {}
for rep in range(a.reps + 1):
    for m16 in ("0", "1"):
        os.environ["RVX_SCAN_M16"] = m16
        rv.synchronize()
        prof = rv.Profiler()
        with prof:
            t0 = time.perf_counter()
            idx.brute_force_device(qb, a.nq, k, ids_b, dist_b)
            rv.synchronize()
            dt = time.perf_counter() - t0
        f = prof.summary().get("scan_filter", {}).get("total_ms", 0.0)
        if rep:  # rep 0 warms both forms
            res.setdefault(m16, []).append((round(dt * 1e3, 2), round(f, 2)))
        out[m16] = (ids_b.download(np.uint64, (a.nq, k)), dist_b.download(np.float32, (a.nq, k)))
        print(f"rep {rep} M16={m16}: call {dt * 1e3:.1f} ms, filter {f:.1f} ms, stats {rv.scan_last_stats()}", flush=True)
same = bool(np.array_equal(out["0"][0], out["1"][0]) and np.array_equal(out["0"][1], out["1"][1]))
flops = 2.0 * a.nq * a.n * a.d
summ = {m: {"call_ms": [c for c, _ in v], "filter_ms": [f for _, f in v],
            "best_filter_frac_of_2500TF": round(flops / (min(f for _, f in v) * 1e-3) / 2.5e15, 4)} for m, v in res.items()}
print(json.dumps({"config": vars(a), "identical": same, "runs": summ}), flush=True)
