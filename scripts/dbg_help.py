import os, sys, numpy as np
sys.path.insert(0, "tests")
import oracle as O
import ruvector_amd as rv
from test_gpu_parity import _sage_stack
os.environ["RVX_SAGE_CHUNKS"] = "2"
n, deg = 40000, 4
d0, d1, d2 = 64, 256, 128
x = O.fill_uniform(n * d0, 60 + n).reshape(n, d0)
rp, col = O.random_csr(n, deg, 61)
g = rv.Graph.from_csr(rp, col)
layers = [rv.GraphSAGELayer(d0, d1, num_samples=deg), rv.GraphSAGELayer(d1, d2, num_samples=deg)]
res = {}
for h in ["0", "1", "2", "1", "2"]:
    os.environ["RVX_SAGE_HELP"] = h[0]
    os.environ["RVX_SAGE_HELP_SYNC"] = "1" if h.endswith("s") else "0"
    for defer in (False, True):
        y1, inv, y2 = _sage_stack(layers, g, x, n, defer)
        key = (h, defer)
        if key in res:
            print("repeat", key, "y1 same", np.array_equal(res[key][0], y1), "inv same", np.array_equal(res[key][1], inv), flush=True)
        res[key] = (y1, inv, y2)
for defer in (False, True):
    a, b = res[("0", defer)], res[("1", defer)]
    bad = np.where(np.any(a[0] != b[0], axis=1))[0]
    badi = np.where(a[1] != b[1])[0]
    print("defer", defer, "y1 rows differ", len(bad), bad[:10], "inv differ", len(badi), badi[:10], flush=True)
for hh in ("1", "2"):
    for defer in (False, True):
        a, b = res[("0", defer)], res[(hh, defer)]
        bad = np.where(np.any(a[0] != b[0], axis=1))[0]
        print("arm", hh, "defer", defer, "rows differ from help0", len(bad), bad[:5], bad[-5:] if len(bad) else "", flush=True)
y1r = res[("0", False)][0]; y1d, inv = res[("0", True)][0], res[("0", True)][1]
e = np.linalg.norm(y1d * inv[:, None] - y1r, axis=1) / np.maximum(np.linalg.norm(y1r, axis=1), 1e-30)
print("help0: worst rows", np.argsort(e)[-5:], e.max(), flush=True)
y1d, inv = res[("1", True)][0], res[("1", True)][1]
y1r = res[("1", False)][0]
e = np.linalg.norm(y1d * inv[:, None] - y1r, axis=1) / np.maximum(np.linalg.norm(y1r, axis=1), 1e-30)
print("help1: worst rows", np.argsort(e)[-5:], e.max(), np.sum(e > 1e-6), flush=True)
