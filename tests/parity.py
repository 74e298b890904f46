"""Parity metrics shared by the GPU tests (and mirrored in bench.py's parity).

North star: "within 1e-5 relative on f32 embeddings". Two readings are checked:
  * normwise:  max|gpu - ref| / max|ref| over the compared block (the embedding's scale);
  * per row:   ||gpu_r - ref_r||_2 / ||ref_r||_2 for every row r with a nonzero
               reference norm; a row whose reference is exactly zero must come out
               within tol of the largest reference row norm (absolute floor).
The per-row bar also bounds every element: |gpu_rj - ref_rj| <= tol * ||ref_r||_2.
"""
import numpy as np


def rel_err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-30)) if b.size else 0.0


def row_rel_err(a, b):
    """max over rows of ||a_r - b_r||_2 / ||b_r||_2 (zero reference rows: / max row norm)."""
    a = np.asarray(a, np.float64).reshape(-1, np.asarray(a).shape[-1] if np.ndim(a) else 1)
    b = np.asarray(b, np.float64).reshape(a.shape)
    if not b.size:
        return 0.0
    nb = np.linalg.norm(b, axis=1)
    nd = np.linalg.norm(a - b, axis=1)
    floor = max(float(nb.max()), 1e-30)
    return float(np.max(nd / np.where(nb > 0, nb, floor)))


def assert_close(a, b, tol=1e-5):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    assert np.all(np.isfinite(a)) == np.all(np.isfinite(b))
    e = rel_err(a, b)
    assert e <= tol, f"normwise relative error {e:.3e} > {tol}"
    r = row_rel_err(a, b)
    assert r <= tol, f"per-row relative error {r:.3e} > {tol}"


def row_rel_vs(a, ref64):
    """Per-row ||a_r - ref_r||_2 / ||ref_r||_2 against an f64 evaluation (vector)."""
    a = np.asarray(a, np.float64)
    nb = np.linalg.norm(ref64, axis=1)
    return np.linalg.norm(a - ref64, axis=1) / np.where(nb > 0, nb, max(float(nb.max()), 1e-30))
