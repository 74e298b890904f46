"""Test infrastructure: the hnsw_rs dump format (patches/hnsw_rs/src/hnswio.rs)
restated in Python — writes a dump of an oracle graph the way
Hnsw::file_dump would (format 4, Full mode; Description::dump :878-919,
PointIndexation::dump :1301-1332, dump_point :1063-1110) and parses a dump
the way load_description / load_point_graph / load_point_indexation read it
(:937-1040, :1221-1290, :615-790). Used to check librvx's native reader and
writer against an independent restatement."""
import math
import struct

import numpy as np

MAGICPOINT, MAGICDESCR_4, MAGICLAYER, MAGICDATAP = 0x000A678F, 0x002A6779, 0x000A676F, 0xA67F0000
NB_LAYER_MAX = 16


def _lists(graph, row):
    """The point's neighbour lists (rows) for layers 0..max_level from an rvx_hnsw_graph dict."""
    out = [list(graph["col0"][graph["row_ptr0"][row]:graph["row_ptr0"][row + 1]])]
    for l in range(1, int(graph["max_level"]) + 1):  # lists above the point's level too
        ids = graph["upper_ids"][l - 1]
        j = int(np.searchsorted(ids, row))
        if j == len(ids) or ids[j] != row:  # a point of this layer whose list is empty
            out.append([])
            continue
        rp = graph["upper_row_ptr"][l - 1]
        out.append(list(graph["upper_col"][l - 1][rp[j]:rp[j + 1]]))
    return out


def write_dump(path_base, graph, vecs, ids, m, ef, distname="anndists::dist::distances::DistL2", dist_fn=None):
    n, d = vecs.shape
    levels = np.asarray(graph["levels"][:n], np.int64)
    rank = np.zeros(n, np.int64)
    by_level = [[] for _ in range(NB_LAYER_MAX)]
    for i in range(n):
        rank[i] = len(by_level[levels[i]])
        by_level[levels[i]].append(i)
    dist_fn = dist_fn or (lambda a, b: float(np.float32(math.sqrt(float(np.sum((a.astype(np.float64) - b) ** 2))))))
    g = bytearray()
    g += struct.pack("<IBBdBQQQ", MAGICDESCR_4, 1, m, 1.0 / math.log(m), NB_LAYER_MAX, ef, n, d)
    for s in (distname.encode(), b"f32"):
        g += struct.pack("<Q", len(s)) + s
    dat = bytearray(struct.pack("<IQ", MAGICDATAP, d))
    g += struct.pack("<B", NB_LAYER_MAX)

    def pid(row):
        return struct.pack("<QBi", int(ids[row]), int(levels[row]), int(rank[row]))

    for l in range(NB_LAYER_MAX):
        g += struct.pack("<IQ", MAGICLAYER, len(by_level[l]))
        for row in by_level[l]:
            g += struct.pack("<I", MAGICPOINT) + pid(row)
            lists = _lists(graph, row)
            for ll in range(NB_LAYER_MAX):
                nb = lists[ll] if ll < len(lists) else []
                g += struct.pack("<Q", len(nb))
                for c in nb:
                    g += pid(c) + struct.pack("<f", dist_fn(vecs[row], vecs[c]))
            dat += struct.pack("<IQQ", MAGICDATAP, int(ids[row]), 4 * d) + np.ascontiguousarray(vecs[row], "<f4").tobytes()
    g += pid(int(graph["entry"]))
    with open(path_base + ".hnsw.graph", "wb") as f:
        f.write(bytes(g))
    with open(path_base + ".hnsw.data", "wb") as f:
        f.write(bytes(dat))


def read_dump(path_base):
    """Parse a Full-mode dump: description, points (origin, layer, rank, lists), entry, vectors."""
    b = open(path_base + ".hnsw.graph", "rb").read()
    o = 0

    def take(fmt):
        nonlocal o
        v = struct.unpack_from("<" + fmt, b, o)
        o += struct.calcsize("<" + fmt)
        return v

    magic, mode, m, scale, nl, ef, npt, dim = take("IBBdBQQQ")
    assert magic == MAGICDESCR_4 and mode == 1
    names = []
    for _ in range(2):
        (ln,) = take("Q")
        names.append(b[o:o + ln].decode())
        o += ln
    (nlay,) = take("B")
    points = []
    for l in range(nlay):
        mg, cnt = take("IQ")
        assert mg == MAGICLAYER
        for r in range(cnt):
            mg, origin, pl, pr = take("IQBi")
            assert mg == MAGICPOINT and pl == l and pr == r
            lists = []
            for _ in range(nl):
                (k,) = take("Q")
                lists.append([take("QBif") for _ in range(k)])
            points.append({"origin": origin, "layer": l, "rank": r, "lists": lists})
    entry = take("QBi")
    assert o == len(b)
    db = open(path_base + ".hnsw.data", "rb").read()
    mg, dd = struct.unpack_from("<IQ", db, 0)
    assert mg == MAGICDATAP and dd == dim
    off, vecs = 12, {}
    for p in points:
        mg, origin, ln = struct.unpack_from("<IQQ", db, off)
        assert mg == MAGICDATAP and origin == p["origin"] and ln == 4 * dim
        vecs[origin] = np.frombuffer(db, "<f4", dim, off + 20).copy()
        off += 20 + ln
    assert off == len(db)
    return {"m": m, "level_scale": scale, "nb_layer": nl, "ef": ef, "nb_point": npt, "dim": dim,
            "distname": names[0], "t_name": names[1], "points": points, "entry": entry, "vectors": vecs}
