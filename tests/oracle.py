"""ctypes wrapper of oracle/liboracle.so — the CPU restatement of the reference.

Test infrastructure only: used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / CPU baseline, never by the
product package (ruvector_amd).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RVX_ORACLE_LIB: the sanitizer build (oracle/_asan/liboracle_asan.so, tests/test_asan.py)
LIB_PATH = os.environ.get("RVX_ORACLE_LIB") or os.path.join(ROOT, "oracle", "liboracle.so")

P, I32, I64, U64, F32 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_float
PF = C.POINTER(C.c_float)
PI64 = C.POINTER(C.c_int64)
PI32 = C.POINTER(C.c_int32)
PU8 = C.POINTER(C.c_uint8)


class Rvl(C.Structure):
    _fields_ = [("in_", C.c_int32), ("H", C.c_int32), ("heads", C.c_int32), ("hd", C.c_int32),
                ("dropout", C.c_float), ("eps", C.c_float)] + [
        (n, PF) for n in ("w_msg", "b_msg", "w_agg", "b_agg", "w_z", "b_wz", "u_z", "b_uz", "w_r", "b_wr", "u_r",
                          "b_ur", "w_h", "b_wh", "u_h", "b_uh", "q", "bq", "k", "bk", "v", "bv", "o", "bo", "gamma",
                          "beta")]


_SIG = {
    "orc_fill_uniform": (None, [PF, I64, U64, F32, F32]),
    "orc_random_csr": (None, [I64, I32, U64, PI64, PI32]),
    "orc_distance": (F32, [PF, PF, I64, I32]),
    "orc_distance_matrix": (None, [PF, I64, PF, I64, I64, I32, PF, I32]),
    "orc_flat_search": (None, [PF, I64, I64, I32, PU8, PF, I64, I32, PI64, PF, I32]),
    "orc_hnsw_new": (P, [I64, I32, I32, I32, I32, U64]),
    "orc_hnsw_free": (None, [P]),
    "orc_hnsw_set_fast": (None, [P, I32]),
    "orc_hnsw_set_lex_stop": (None, [P, I32]),
    "orc_simd_width": (I32, []),
    "orc_flat_search_fast": (None, [PF, I64, I64, I32, PF, I64, I32, PI64, PF, I32]),
    "orc_hnsw_insert": (None, [P, PF, I64, I32]),
    "orc_hnsw_search": (None, [P, PF, I64, I32, I32, PI64, PF, PI32, I32]),
    "orc_hnsw_export_sizes": (None, [P, PI64, PI32, PI64, PI64, PI64, PI64]),
    "orc_hnsw_export": (None, [P, PU8, PI64, PI32, PF, PI32, PI64, PI32]),
    "orc_hnsw_from_graph": (P, [PF, I64, I64, I32, PU8, I64, I32, PI64, PI32, PI64, PI32, PI64, PI32]),
    "orc_sage_init": (None, [I32, I32, I32, PF]),
    "orc_build_csr": (I64, [I64, PI64, PI64, I64, PF, PI64, PI32, PF]),
    "orc_aggregate": (None, [PF, I64, I32, PI64, PI32, PF, I32, I32, PF]),
    "orc_sage_forward": (None, [PF, I64, I32, I32, PI64, PI32, PF, PF, I32, I32, I64, I64, PF, I32, I32]),
    "orc_sage_sample_positions": (None, [I32, I32, PI32]),
    "orc_chacha_words": (None, [C.POINTER(C.c_uint32), I32, I32, C.POINTER(C.c_uint32)]),
    "orc_gcn_forward": (None, [PF, I64, I32, I32, PI64, PI32, PF, PF, PF, I32, PF, I32]),
    "orc_rvl_forward_one": (None, [C.POINTER(Rvl), PF, PF, I32, PF, I32, PF]),
    "orc_rvl_forward_graph": (None, [C.POINTER(Rvl), PF, I64, PI64, PI32, PF, I64, I64, PF, I32]),
    "orc_cosine_similarity": (F32, [PF, PF, I64]),
    "orc_differentiable_search": (I32, [PF, PF, I32, I64, I32, F32, PI64, PF]),
    "orc_hierarchical_forward": (I32, [P, I32, P, PI64, I32, PF, I32, PF]),
    "orc_efa_init": (None, [I32, I32, I32, PF, PF, PF, PF, PF]),
    "orc_dsa_init": (None, [I32, PF, PF, PF]),
    "orc_dsa_compute": (I32, [I32, F32, F32, F32, F32, PF, PF, PF, PF, PF, PF, I32, I32, PF]),
    "orc_efa_compute": (I32, [I32, I32, I32, I32, F32, PF, PF, PF, PF, PF, PF, PF, PF, PF, I32, PF]),
    "orc_poincare_distance": (F32, [PF, PF, I64, F32]),
    "orc_hyp_new": (P, [I32, I32, I32, I32, I32, F32, F32, I32, U64]),
    "orc_hyp_free": (None, [P]),
    "orc_hyp_len": (I64, [P]),
    "orc_hyp_insert": (None, [P, PF, I64]),
    "orc_hyp_get_vector": (None, [P, I64, PF]),
    "orc_hyp_search": (None, [P, PF, I64, I32, I32, PI64, PF, PI32, I32]),
    "orc_hyp_brute_force": (None, [P, PF, I64, I32, PI64, PF, I32]),
    "orc_hyp_build_tangent": (None, [P]),
    "orc_hyp_centroid": (None, [P, PF]),
    "orc_hyp_scan_rows": (None, [PF, I64, I32, F32, PF, I64, I32, I64, PI64, PF, I32]),
    "orc_libm_check": (I64, [I32, U64, U64, U64, PF, I32, C.POINTER(C.c_uint32)]),
    "orc_hyp_search_pruning": (None, [P, PF, I64, I32, PI64, PF, I32]),
    "orc_hyp_set_curvature": (None, [P, F32]),
    "orc_hyp_set_metric": (None, [P, I32]),
    "orc_hyp_export_sizes": (None, [P, PI64, PI32, PI64, PI64, PI64, PI64]),
    "orc_hyp_export": (None, [P, PU8, PI64, PI32, PI32, PI64, PI32]),
    "orc_hyp_from_graph": (P, [PF, I64, I32, I32, I32, I32, F32, I32, PU8, I64, I32, PI64, PI32, PI64, PI32, PI64,
                               PI32]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
        l = C.CDLL(LIB_PATH)
        for n, (r, a) in _SIG.items():
            f = getattr(l, n)
            f.restype = r
            f.argtypes = a
        _lib = l
    return _lib


def fp(a):
    return a.ctypes.data_as(PF) if a is not None else None


def ip64(a):
    return a.ctypes.data_as(PI64) if a is not None else None


def ip32(a):
    return a.ctypes.data_as(PI32) if a is not None else None


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


METRICS = {"l2": 0, "cosine": 1, "dot": 2, "l1": 3}


def fill_uniform(n, seed, lo=-1.0, hi=1.0):
    out = np.empty(n, np.float32)
    lib().orc_fill_uniform(fp(out), n, seed, lo, hi)
    return out


def random_csr(n, deg, seed):
    rp = np.empty(n + 1, np.int64)
    col = np.empty(max(n * deg, 1), np.int32)
    lib().orc_random_csr(n, deg, seed, ip64(rp), ip32(col))
    return rp, col[:n * deg]


def distance(a, b, metric="l2"):
    a, b = f32(a), f32(b)
    return lib().orc_distance(fp(a), fp(b), a.size, METRICS[metric])


def distance_matrix(q, x, metric="l2", threads=8):
    q, x = f32(q), f32(x)
    out = np.empty((q.shape[0], x.shape[0]), np.float32)
    lib().orc_distance_matrix(fp(q), q.shape[0], fp(x), x.shape[0], q.shape[1], METRICS[metric], fp(out), threads)
    return out


def flat_search(base, q, k, metric="l2", deleted=None, threads=8):
    base, q = f32(base), f32(q)
    ids = np.empty((q.shape[0], k), np.int64)
    d = np.empty((q.shape[0], k), np.float32)
    dl = None if deleted is None else np.ascontiguousarray(deleted, np.uint8)
    lib().orc_flat_search(fp(base), base.shape[0], base.shape[1], METRICS[metric],
                          dl.ctypes.data_as(PU8) if dl is not None else None, fp(q), q.shape[0], k, ip64(ids), fp(d),
                          threads)
    return ids, d


class Hnsw:
    """hnsw_rs 0.3.3 as wired by ruvector-core HnswIndex (max_layer = min(16, dim))."""

    def __init__(self, dim, metric="l2", m=32, ef_construction=200, seed=1, max_layer=None, _h=None):
        self.dim = dim
        self.metric = metric
        self._h = _h or lib().orc_hnsw_new(dim, METRICS[metric], m, ef_construction,
                                            min(16, dim) if max_layer is None else max_layer, seed)

    def insert(self, vecs, threads=8):
        v = f32(vecs)
        lib().orc_hnsw_insert(self._h, fp(v), v.shape[0], threads)

    def search(self, q, k, ef, threads=8, lex_stop=True):
        """lex_stop False: the reference's distance-only stop test (hnsw.rs:913-1055)
        instead of the (d, id) rule the GPU search shares."""
        q = f32(q)
        nq = q.shape[0]
        ids = np.empty((nq, k), np.int64)
        d = np.empty((nq, k), np.float32)
        cnt = np.empty(nq, np.int32)
        lib().orc_hnsw_set_lex_stop(self._h, int(bool(lex_stop)))
        lib().orc_hnsw_search(self._h, fp(q), nq, k, ef, ip64(ids), fp(d), ip32(cnt), threads)
        lib().orc_hnsw_set_lex_stop(self._h, 1)
        return ids, d, cnt

    def export(self):
        n, ml, ent, e0 = C.c_int64(), C.c_int32(), C.c_int64(), C.c_int64()
        uc = np.zeros(17, np.int64)
        ue = np.zeros(17, np.int64)
        lib().orc_hnsw_export_sizes(self._h, C.byref(n), C.byref(ml), C.byref(ent), C.byref(e0), ip64(uc), ip64(ue))
        N, L = n.value, ml.value
        levels = np.empty(max(N, 1), np.uint8)
        rp0 = np.empty(N + 1, np.int64)
        col0 = np.empty(max(e0.value, 1), np.int32)
        dist0 = np.empty(max(e0.value, 1), np.float32)
        tot_ids = int(uc[1:L + 1].sum())
        tot_rp = int((uc[1:L + 1] + 1).sum())
        tot_col = int(ue[1:L + 1].sum())
        up_ids = np.empty(max(tot_ids, 1), np.int32)
        up_rp = np.empty(max(tot_rp, 1), np.int64)
        up_col = np.empty(max(tot_col, 1), np.int32)
        lib().orc_hnsw_export(self._h, levels.ctypes.data_as(PU8), ip64(rp0), ip32(col0), fp(dist0), ip32(up_ids),
                              ip64(up_rp), ip32(up_col))
        g = {"n": N, "max_level": L, "entry": ent.value, "levels": levels[:N], "row_ptr0": rp0,
             "col0": col0[:e0.value], "dist0": dist0[:e0.value], "upper_ids": [], "upper_row_ptr": [],
             "upper_col": []}
        oi = orp = oc = 0
        for l in range(1, L + 1):
            c = int(uc[l])
            g["upper_ids"].append(up_ids[oi:oi + c].copy())
            rp = up_rp[orp:orp + c + 1].copy()
            g["upper_row_ptr"].append(rp)
            g["upper_col"].append(up_col[oc:oc + int(rp[-1])].copy())
            oi += c
            orp += c + 1
            oc += int(rp[-1])
        return g

    @classmethod
    def from_graph(cls, vecs, g, metric="l2"):
        v = f32(vecs)
        L = g["max_level"]
        uc = np.zeros(17, np.int64)
        for l in range(1, L + 1):
            uc[l] = len(g["upper_ids"][l - 1])
        cat32 = lambda xs: np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros(1), np.int32)  # noqa: E731
        cat64 = lambda xs: np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros(1), np.int64)  # noqa: E731
        ids, rps, cols = cat32(g["upper_ids"]), cat64(g["upper_row_ptr"]), cat32(g["upper_col"])
        lv = np.ascontiguousarray(g["levels"], np.uint8)
        rp0 = np.ascontiguousarray(g["row_ptr0"], np.int64)
        col0 = np.ascontiguousarray(g["col0"], np.int32)
        h = lib().orc_hnsw_from_graph(fp(v), v.shape[0], v.shape[1], METRICS[metric], lv.ctypes.data_as(PU8),
                                      g["entry"], L, ip64(rp0), ip32(col0), ip64(uc), ip32(ids), ip64(rps), ip32(cols))
        return cls(v.shape[1], metric, _h=h)

    def __del__(self):
        try:
            lib().orc_hnsw_free(self._h)
        except Exception:
            pass


def sage_init(in_f, out_f, offset):
    w = np.empty((in_f, out_f), np.float32)
    lib().orc_sage_init(in_f, out_f, offset, fp(w))
    return w


def build_csr(n, edge_index, weights=None):
    ei = np.asarray(edge_index, dtype=np.int64).reshape(-1, 2)
    src, dst = np.ascontiguousarray(ei[:, 0]), np.ascontiguousarray(ei[:, 1])
    rp = np.empty(n + 1, np.int64)
    col = np.empty(max(len(src), 1), np.int32)
    w = None if weights is None else f32(weights)
    wo = np.empty(max(len(src), 1), np.float32)
    e = lib().orc_build_csr(n, ip64(src), ip64(dst), len(src), fp(w), ip64(rp), ip32(col), fp(wo))
    return rp, col[:e], (wo[:e] if w is not None else None)


def aggregate(x, rp, col, method="sum", w=None, keep_isolated=False):
    x = f32(x)
    n, dim = x.shape
    out = np.empty_like(x)
    m = {"sum": 0, "mean": 1, "max": 2}[method]
    lib().orc_aggregate(fp(x), n, dim, ip64(np.ascontiguousarray(rp, np.int64)),
                        ip32(np.ascontiguousarray(col, np.int32)), fp(None if w is None else f32(w)), m,
                        int(keep_isolated), fp(out))
    return out


def sage_forward(x, rp, col, wn, ws, aggregator=0, normalize=True, rows=None, threads=8, num_samples=None):
    x, wn, ws = f32(x), f32(wn), f32(ws)
    n, in_f = x.shape
    out_f = wn.shape[1]
    r0, nr = (0, n) if rows is None else rows
    y = np.empty((nr, out_f), np.float32)
    lib().orc_sage_forward(fp(x), n, in_f, out_f, ip64(np.ascontiguousarray(rp, np.int64)),
                           ip32(np.ascontiguousarray(col, np.int32)), fp(wn), fp(ws), aggregator, int(normalize), r0,
                           nr, fp(y), threads, 2**31 - 1 if num_samples is None else int(num_samples))
    return y


def sage_sample_positions(length, k):
    """Positions GraphSAGELayer::sample_neighbors keeps for a list of `length` > k (graphsage.rs:92-102)."""
    out = np.empty(k, np.int32)
    lib().orc_sage_sample_positions(int(length), int(k), ip32(out))
    return out


def chacha_words(key_words, rounds, nwords):
    """ChaCha keystream (block 0 on, zero nonce) — the rand_chacha core of StdRng."""
    key = np.ascontiguousarray(key_words, np.uint32)
    out = np.empty(nwords, np.uint32)
    lib().orc_chacha_words(key.ctypes.data_as(C.POINTER(C.c_uint32)), int(rounds), int(nwords),
                           out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out


def gcn_forward(x, rp, col, w, bias=None, ew=None, normalize=True, threads=8):
    x, w = f32(x), f32(w)
    n, in_f = x.shape
    out_f = w.shape[1]
    y = np.zeros((n, out_f), np.float32)
    lib().orc_gcn_forward(fp(x), n, in_f, out_f, ip64(np.ascontiguousarray(rp, np.int64)),
                          ip32(np.ascontiguousarray(col, np.int32)), fp(None if ew is None else f32(ew)), fp(w),
                          fp(None if bias is None else f32(bias)), int(normalize), fp(y), threads)
    return y


class RvlWeights:
    """RuvectorLayer weights parsed from its serde JSON (layer.rs:313-333)."""

    def __init__(self, js: dict):
        def lin(o):
            w = np.asarray(o["weights"]["data"], np.float32).reshape(o["weights"]["dim"])
            b = np.asarray(o["bias"]["data"], np.float32)
            return np.ascontiguousarray(w), np.ascontiguousarray(b)
        self.arrays = {}
        for name, obj in (("msg", js["w_msg"]), ("agg", js["w_agg"]), ("z", js["w_update"]["w_z"]),
                          ("uz", js["w_update"]["u_z"]), ("r", js["w_update"]["w_r"]), ("ur", js["w_update"]["u_r"]),
                          ("h", js["w_update"]["w_h"]), ("uh", js["w_update"]["u_h"]),
                          ("q", js["attention"]["q_linear"]), ("k", js["attention"]["k_linear"]),
                          ("v", js["attention"]["v_linear"]), ("o", js["attention"]["out_linear"])):
            self.arrays[name] = lin(obj)
        self.gamma = np.asarray(js["norm"]["gamma"]["data"], np.float32)
        self.beta = np.asarray(js["norm"]["beta"]["data"], np.float32)
        A = self.arrays
        self.s = Rvl(in_=A["msg"][0].shape[1], H=A["msg"][0].shape[0], heads=js["attention"]["num_heads"],
                     hd=js["attention"]["head_dim"], dropout=js["dropout"], eps=js["norm"]["eps"],
                     w_msg=fp(A["msg"][0]), b_msg=fp(A["msg"][1]), w_agg=fp(A["agg"][0]), b_agg=fp(A["agg"][1]),
                     w_z=fp(A["z"][0]), b_wz=fp(A["z"][1]), u_z=fp(A["uz"][0]), b_uz=fp(A["uz"][1]),
                     w_r=fp(A["r"][0]), b_wr=fp(A["r"][1]), u_r=fp(A["ur"][0]), b_ur=fp(A["ur"][1]),
                     w_h=fp(A["h"][0]), b_wh=fp(A["h"][1]), u_h=fp(A["uh"][0]), b_uh=fp(A["uh"][1]),
                     q=fp(A["q"][0]), bq=fp(A["q"][1]), k=fp(A["k"][0]), bk=fp(A["k"][1]), v=fp(A["v"][0]),
                     bv=fp(A["v"][1]), o=fp(A["o"][0]), bo=fp(A["o"][1]), gamma=fp(self.gamma), beta=fp(self.beta))
        self.H = self.s.H
        self.in_dim = self.s.in_


def rvl_forward_one(W: RvlWeights, node, nbrs, weights):
    node = f32(node).reshape(-1)
    deg = len(nbrs)
    nb = f32(nbrs).reshape(deg, -1) if deg else np.zeros((1, W.in_dim), np.float32)
    w = f32(weights).reshape(-1) if len(weights) else np.zeros(1, np.float32)
    out = np.empty(W.H, np.float32)
    lib().orc_rvl_forward_one(C.byref(W.s), fp(node), fp(nb), deg, fp(w), len(weights), fp(out))
    return out


def rvl_forward_graph(W: RvlWeights, x, rp, col, ew=None, rows=None, threads=8):
    x = f32(x)
    n = x.shape[0]
    r0, nr = (0, n) if rows is None else rows
    y = np.empty((nr, W.H), np.float32)
    lib().orc_rvl_forward_graph(C.byref(W.s), fp(x), n, ip64(np.ascontiguousarray(rp, np.int64)),
                                ip32(np.ascontiguousarray(col, np.int32)), fp(None if ew is None else f32(ew)), r0, nr,
                                fp(y), threads)
    return y


def cosine_similarity(a, b):
    a, b = f32(a), f32(b)
    return lib().orc_cosine_similarity(fp(a), fp(b), a.size)


def differentiable_search(q, cand, k, temperature):
    q, cand = f32(q), f32(cand)
    c = cand.shape[0] if cand.size else 0
    idx = np.empty(max(k, 1), np.int64)
    w = np.empty(max(k, 1), np.float32)
    n = lib().orc_differentiable_search(fp(q), fp(cand) if c else None, c, q.size, k, temperature, ip64(idx), fp(w))
    return idx[:n], w[:n]


def hierarchical_forward(q, levels, weights):
    """hierarchical_forward (search.rs:105-162), one query; levels: list of [rows][dim]
    arrays, weights: list of RvlWeights (zip of the two)."""
    q = f32(q).reshape(-1)
    nl, nv = len(weights), len(levels)
    lv = [f32(np.asarray(e, np.float32).reshape(len(e), -1)) if len(e) else np.zeros((0, 1), np.float32) for e in levels]
    lay = (C.c_void_p * max(nl, 1))(*[C.cast(C.byref(W.s), C.c_void_p).value for W in weights])
    lev = (C.c_void_p * max(nv, 1))(*[e.ctypes.data if e.size else None for e in lv])
    rows = np.ascontiguousarray([len(e) for e in lv] or [0], dtype=np.int64)
    out = np.empty(max([q.size] + [W.H for W in weights]), np.float32)
    n = lib().orc_hierarchical_forward(lay, nl, lev, ip64(rows), nv, fp(q), q.size, fp(out))
    return out[:n].copy()


def efa_init(node_dim, edge_dim, heads):
    hd = node_dim // heads
    wn = np.empty(heads * hd * node_dim, np.float32)
    we = np.empty(max(heads * hd * edge_dim, 1), np.float32)
    a_s, a_d, a_e = (np.empty(heads * hd, np.float32) for _ in range(3))
    lib().orc_efa_init(node_dim, edge_dim, heads, fp(wn), fp(we), fp(a_s), fp(a_d), fp(a_e))
    return wn, we, a_s, a_d, a_e


def efa_compute(node_dim, edge_dim, heads, query, keys, values, edges=None, concat=True, slope=0.2):
    wn, we, a_s, a_d, a_e = efa_init(node_dim, edge_dim, heads)
    q = f32(query)
    n = len(keys)
    k = f32(keys).reshape(n, node_dim) if n else np.zeros((1, node_dim), np.float32)
    v = f32(values).reshape(n, node_dim) if n else np.zeros((1, node_dim), np.float32)
    e = None if edges is None else (f32(edges).reshape(n, edge_dim) if n and edge_dim else np.zeros((1, 1), np.float32))
    out = np.empty(node_dim, np.float32)
    m = lib().orc_efa_compute(node_dim, edge_dim, heads, int(concat), slope, fp(wn), fp(we), fp(a_s), fp(a_d),
                              fp(a_e), fp(q), fp(k), fp(v), fp(e), n, fp(out))
    return out[:m]


def dsa_init(dim):
    """DualSpaceAttention::new weights (dual_space.rs:107-131): w_euclidean, w_hyperbolic, w_out [dim][dim]."""
    w = [np.empty(dim * dim, np.float32) for _ in range(3)]
    lib().orc_dsa_init(dim, fp(w[0]), fp(w[1]), fp(w[2]))
    return w


def dsa_compute(dim, query, keys, values, curvature=1.0, euclidean_weight=0.5, hyperbolic_weight=0.5,
                temperature=1.0):
    """DualSpaceAttention::compute (dual_space.rs:207-268); None for empty keys (the reference's Err)."""
    we, wh, wo = dsa_init(dim)
    q = f32(query)
    n = len(keys)
    if n == 0:
        return None
    k = f32(keys).reshape(n, dim)
    v = f32(values).reshape(n, -1)
    out = np.empty(max(v.shape[1], dim), np.float32)
    m = lib().orc_dsa_compute(dim, curvature, euclidean_weight, hyperbolic_weight, temperature, fp(we), fp(wh),
                              fp(wo), fp(q), fp(k), fp(v), n, v.shape[1], fp(out))
    return out[:m]


def poincare_distance(u, v, c=1.0):
    u, v = f32(u), f32(v)
    return lib().orc_poincare_distance(fp(u), fp(v), u.size, c)


class Hyp:
    """HyperbolicHnsw restated (oracle/hyperbolic.cpp; crates/ruvector-hyperbolic-hnsw/src/hnsw.rs)."""

    def __init__(self, dim, m=16, m0=32, ef_construction=200, ef_search=50, level_mult=None, curvature=1.0,
                 prune_factor=10, seed=0, _h=None):
        import math
        self.dim = dim
        lm = 1.0 / math.log(16.0) if level_mult is None else level_mult
        self._h = _h or lib().orc_hyp_new(dim, m, m0, ef_construction, ef_search, lm, curvature, prune_factor, seed)

    def __len__(self):
        return lib().orc_hyp_len(self._h)

    def insert(self, vecs):
        v = f32(vecs).reshape(-1, self.dim)
        lib().orc_hyp_insert(self._h, fp(v), v.shape[0])

    def get_vector(self, i):
        out = np.empty(self.dim, np.float32)
        lib().orc_hyp_get_vector(self._h, int(i), fp(out))
        return out

    def _q(self, q, k):
        q = f32(q).reshape(-1, self.dim)
        return q, np.empty((q.shape[0], k), np.int64), np.empty((q.shape[0], k), np.float32)

    def search(self, q, k, ef=0, threads=8):
        q, ids, d = self._q(q, k)
        cnt = np.empty(q.shape[0], np.int32)
        lib().orc_hyp_search(self._h, fp(q), q.shape[0], k, ef, ip64(ids), fp(d), ip32(cnt), threads)
        return ids, d, cnt

    def brute_force(self, q, k, threads=8):
        q, ids, d = self._q(q, k)
        lib().orc_hyp_brute_force(self._h, fp(q), q.shape[0], k, ip64(ids), fp(d), threads)
        return ids, d

    def build_tangent_cache(self):
        lib().orc_hyp_build_tangent(self._h)

    def centroid(self):
        out = np.empty(self.dim, np.float32)
        lib().orc_hyp_centroid(self._h, fp(out))
        return out

    def search_with_pruning(self, q, k, threads=8):
        q, ids, d = self._q(q, k)
        lib().orc_hyp_search_pruning(self._h, fp(q), q.shape[0], k, ip64(ids), fp(d), threads)
        return ids, d

    def set_curvature(self, c):
        lib().orc_hyp_set_curvature(self._h, float(c))

    def set_metric(self, metric):
        """'poincare' or 'euclidean' (HyperbolicHnswConfig.metric, hnsw.rs:23-32)."""
        lib().orc_hyp_set_metric(self._h, 1 if metric == "euclidean" else 0)

    def export(self):
        n, ml, ent, e0 = C.c_int64(), C.c_int32(), C.c_int64(), C.c_int64()
        uc = np.zeros(17, np.int64)
        ue = np.zeros(17, np.int64)
        lib().orc_hyp_export_sizes(self._h, C.byref(n), C.byref(ml), C.byref(ent), C.byref(e0), ip64(uc), ip64(ue))
        N, L = n.value, ml.value
        levels = np.empty(max(N, 1), np.uint8)
        rp0 = np.empty(N + 1, np.int64)
        col0 = np.empty(max(e0.value, 1), np.int32)
        up_ids = np.empty(max(int(uc[1:L + 1].sum()), 1), np.int32)
        up_rp = np.empty(max(int((uc[1:L + 1] + 1).sum()), 1), np.int64)
        up_col = np.empty(max(int(ue[1:L + 1].sum()), 1), np.int32)
        lib().orc_hyp_export(self._h, levels.ctypes.data_as(PU8), ip64(rp0), ip32(col0), ip32(up_ids), ip64(up_rp),
                             ip32(up_col))
        g = {"n": N, "max_level": L, "entry": ent.value, "levels": levels[:N], "row_ptr0": rp0,
             "col0": col0[:e0.value], "upper_ids": [], "upper_row_ptr": [], "upper_col": []}
        oi = orp = oc = 0
        for l in range(1, L + 1):
            c = int(uc[l])
            g["upper_ids"].append(up_ids[oi:oi + c].copy())
            rp = up_rp[orp:orp + c + 1].copy()
            g["upper_row_ptr"].append(rp)
            g["upper_col"].append(up_col[oc:oc + int(rp[-1])].copy())
            oi += c
            orp += c + 1
            oc += int(rp[-1])
        return g

    @classmethod
    def from_graph(cls, vecs, g, m=16, m0=32, ef_search=50, curvature=1.0, prune_factor=10):
        v = f32(vecs)
        L = g["max_level"]
        uc = np.zeros(17, np.int64)
        for l in range(1, L + 1):
            uc[l] = len(g["upper_ids"][l - 1])
        cat32 = lambda xs: np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros(1), np.int32)  # noqa: E731
        cat64 = lambda xs: np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros(1), np.int64)  # noqa: E731
        ids, rps, cols = cat32(g["upper_ids"]), cat64(g["upper_row_ptr"]), cat32(g["upper_col"])
        lv = np.ascontiguousarray(g["levels"], np.uint8)
        h = lib().orc_hyp_from_graph(fp(v), v.shape[0], v.shape[1], m, m0, ef_search, curvature, prune_factor,
                                     lv.ctypes.data_as(PU8), g["entry"], L, ip64(np.ascontiguousarray(g["row_ptr0"],
                                                                                                       np.int64)),
                                     ip32(np.ascontiguousarray(g["col0"], np.int32)), ip64(uc), ip32(ids), ip64(rps),
                                     ip32(cols))
        return cls(v.shape[1], _h=h)

    def __del__(self):
        try:
            lib().orc_hyp_free(self._h)
        except Exception:
            pass


def dual_space_search(hyp, euc, query, k, fusion_weight, curvature=1.0):
    """DualSpaceIndex::search (crates/ruvector-hyperbolic-hnsw/src/hnsw.rs:573-605) over two
    oracle Hyp indexes (Poincaré and Euclidean metric): 2k from each, f32 reciprocal-rank
    fusion, highest score first (ties by first appearance), Poincaré distance of the raw
    query to the stored vector. Returns [(id, distance)]."""
    q = f32(query).reshape(1, -1)
    hi, _, hc = hyp.search(q, 2 * k)
    ei, _, ec = euc.search(q, 2 * k)
    w = np.float32(min(max(fusion_weight, 0.0), 1.0))
    scores = {}
    for rank, i in enumerate(hi[0][:hc[0]]):
        scores[int(i)] = np.float32(scores.get(int(i), np.float32(0.0)) + w * (np.float32(1.0) / np.float32(rank + 1)))
    for rank, i in enumerate(ei[0][:ec[0]]):
        scores[int(i)] = np.float32(scores.get(int(i), np.float32(0.0)) +
                                    (np.float32(1.0) - w) * (np.float32(1.0) / np.float32(rank + 1)))
    top = sorted(scores.items(), key=lambda t: -t[1])[:k]
    return [(i, poincare_distance(q[0], hyp.get_vector(i), curvature)) for i, _ in top]


LIBM_FNS = ("logf", "log1pf", "expm1f", "tanhf", "atanh")


def libm_check(fn, start=0, stride=1, count=1 << 32, dev=None, threads=None):
    """Mismatches of the libm restatements (ruvector_amd/csrc/libm_f32.hpp) against the
    host glibc over x = bits(start + i*stride), i < count: the host-compiled restatement
    when dev is None, else the device outputs dev[i]. Returns (mismatches, first bad bits)."""
    fb = C.c_uint32()
    threads = threads or min(16, os.cpu_count() or 8)
    dev = None if dev is None else np.ascontiguousarray(dev, np.float32)
    ptr = None if dev is None else fp(dev)
    bad = lib().orc_libm_check(LIBM_FNS.index(fn), start, stride, count, ptr, threads, C.byref(fb))
    return int(bad), int(fb.value)


def hyp_scan_rows(x, q, k, id_base=0, ids=None, dist=None, c=1.0, threads=8):
    """Merge the exact Poincaré top-k of rows x (ids id_base + i) into (ids, dist)
    (orc_hyp_scan_rows); start from ids=None for a fresh scan."""
    x, q = f32(x), f32(q)
    nq = q.shape[0]
    if ids is None:
        ids, dist = np.full((nq, k), -1, np.int64), np.full((nq, k), np.inf, np.float32)
    lib().orc_hyp_scan_rows(fp(x), x.shape[0], x.shape[1], c, fp(q), nq, k, id_base, ip64(ids), fp(dist), threads)
    return ids, dist
