import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import oracle as O, ruvector_amd as rv
n, d, deg = 400_000, 64, 8
x = rv.Buffer(n * d * 4); x.fill_uniform(n * d, 21, -1.0, 1.0)
g = rv.Graph.random(n, deg, 22)
layer = rv.GraphSAGELayer(d, d, num_samples=deg)
y = rv.Buffer(n * d * 4); layer.forward_device(x, g, y)
got = y.download(np.float32, (n, d)); xs = x.download(np.float32, (n, d))
rp, col = O.random_csr(n, deg, 22)
wn, ws = O.sage_init(d, d, 0), O.sage_init(d, d, 1000)
for r0 in (0, 16_768 - 1500, n - 3000):
    ref = O.sage_forward(xs, rp, col, wn, ws, rows=(r0, 3000))
    a = got[r0:r0 + 3000].astype(np.float64); b = ref.astype(np.float64)
    diff = np.abs(a - b); i, j = np.unravel_index(np.argmax(diff), diff.shape)
    print(r0, "rel", diff.max() / np.abs(b).max(), "row", r0 + i, "nnz", int((b[i] != 0).sum()), "rowmax", np.abs(b[i]).max(),
          "row err/rowmax", diff[i].max() / np.abs(b[i]).max())
import os
os.environ["RVX_GEMM_H2"] = "0"
y2 = rv.Buffer(n * d * 4); layer.forward_device(x, g, y2)
got2 = y2.download(np.float32, (n, d))
for r0 in (0, 16_768 - 1500, n - 3000):
    ref = O.sage_forward(xs, rp, col, wn, ws, rows=(r0, 3000))
    print("x3", r0, np.abs(got2[r0:r0+3000].astype(np.float64) - ref).max() / np.abs(ref).max())
