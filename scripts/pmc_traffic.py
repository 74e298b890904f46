#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into per-kernel HBM bytes.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per
128-B request of a wide coalesced stream, i.e. half the bytes read, so the
read side is doubled; WRITE_SIZE is exact for 16-B-per-lane stores. Both
counters are in KiB. Usage:
  pmc_traffic.py <fetch_dir> <write_dir> <out.json>
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

TAGS = {  # kernel symbol substring -> bench tag
    # the overlapped gather takes its rows from a counter (RVX_SAGE_HELP=1) and the previous
    # chunk's GEMM takes some of them: its bytes are split between the two kernels, so the pair
    # is also reported per chunk (sage_chunk_gather_gemm); the static gathers are the bench's
    # gemm_paths alternatives (no help)
    "k_aggregate_help": "sage_aggregate",
    "k_aggregate_vec": "sage_aggregate_static",
    # one entry per GEMM kernel: the layer's split-f16 GEMM (h2g) alone under sage_gemm; the
    # alternatives bench.py times (gemm_paths) under their own names
    "gemm_nt_h2g": "sage_gemm",
    "gemm_nt_h2w": "sage_gemm",
    "gemm_nt_x3": "sage_gemm_alt_split_bf16x6",
    "gemm_nt_mfma": "sage_gemm_alt_fp32_mfma",
    "k_normalize_rows": "sage_normalize",
    "k_scan_topk": "scan_topk",
    "k_scan_filter": "scan_filter",
    "k_rows_to_f16": "scan_f16",
    "k_hnsw_search": "hnsw_search",
    "k_edge_attn": "gnn_edge_attention",
    "k_rows_image_pack": "rows_image_pack",
}


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: [0.0, set()])
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                acc[name][0] += float(row["Counter_Value"])
                acc[name][1].add(disp)
    return {k: (v[0], len(v[1])) for k, v in acc.items()}


# C4 stack (bench_gnn.py): the RuvectorLayer GEMMs are the split-f16 h2w tiles (the attention
# head's transform runs split-bf16 x3g, its own tag), the edge kernel k_edge_attn_grouped
TAGS_C4 = {
    "gemm_nt_h2w": "gnn_gemm",
    "gemm_nt_h2g": "gnn_gemm",
    "k_edge_attn": "gnn_edge_attention",
    "k_gru_finish": "gnn_finish",
    "k_mul_amax": "gnn_gate",
    "gemm_nt_x3g": "efa_gemm",
    "k_edge_feat": "efa_edge",
}


def load_dispatches(d, counter, substr):
    """Per-dispatch counter totals of the kernels whose name contains substr, in dispatch order."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(float)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter or substr not in row.get("Kernel_Name", ""):
                    continue
                acc[int(row.get("Dispatch_Id") or row.get("Correlation_Id"))] += float(row["Counter_Value"])
    return [acc[k] for k in sorted(acc)]


def main_c3():
    """bench_c3.py under --pmc: the hnsw_search dispatches run in the order warm / timed per ef of
    the sweep, then NeuralSearch's warm-up and timed searches; the timed launch of sweep entry i
    is dispatch 2 i + 1. Usage: pmc_traffic.py --c3 <fetch_dir> <write_dir> <out.json> <bench.json>"""
    fdir, wdir, out, bj = sys.argv[1:5]
    j = json.loads([l for l in open(bj) if l.startswith("{")][-1])
    fetch = load_dispatches(fdir, "FETCH_SIZE", "k_hnsw_search")
    write = load_dispatches(wdir, "WRITE_SIZE", "k_hnsw_search")
    by_ef = {}
    for i, s in enumerate(j["sweep"]):
        t = 2 * i + 1
        if t < len(fetch) and t < len(write):
            rd, wr = 2.0 * fetch[t] * 1024, write[t] * 1024
            by_ef[str(s["ef"])] = {"read_bytes_per_launch_corrected": rd, "write_bytes_per_launch": wr,
                                   "hbm_bytes_per_launch": rd + wr,
                                   "alg_bytes_per_launch": s["roofline"]["alg_bytes_per_launch"]}
    cfg = j.get("c3_config") or {}
    json.dump({"config": cfg, "kernels": {"hnsw_search_by_ef": by_ef}, "dispatches": len(fetch)}, open(out, "w"),
              indent=1)
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e9, 2) for k, v in by_ef.items()}))


def main():
    if "--c3" in sys.argv:
        sys.argv.remove("--c3")
        return main_c3()
    tags = TAGS
    if "--c4" in sys.argv:
        sys.argv.remove("--c4")
        tags = TAGS_C4
    fdir, wdir, out = sys.argv[1:4]
    fetch = load(fdir, "FETCH_SIZE")
    write = load(wdir, "WRITE_SIZE")
    res = {}
    for name in set(fetch) | set(write):
        tag = next((t for s, t in tags.items() if s in name), None)
        if tag is None:
            continue
        fk, fn = fetch.get(name, (0.0, 0))
        wk, wn = write.get(name, (0.0, 0))
        ent = res.setdefault(tag, {"kernels": [], "fetch_kib": 0.0, "write_kib": 0.0, "fetch_n": 0, "write_n": 0})
        ent["kernels"].append(re.sub(r"\s+", " ", name)[:120])
        ent["fetch_kib"] += fk
        ent["write_kib"] += wk
        ent["fetch_n"] += fn
        ent["write_n"] += wn
    for tag, e in res.items():
        rd = 2.0 * e["fetch_kib"] * 1024 / max(e["fetch_n"], 1)
        wr = e["write_kib"] * 1024 / max(e["write_n"], 1)
        e["read_bytes_per_launch_corrected"] = rd
        e["write_bytes_per_launch"] = wr
        e["hbm_bytes_per_launch"] = rd + wr
        e["hbm_bytes_total"] = 2.0 * e["fetch_kib"] * 1024 + e["write_kib"] * 1024
    if "sage_aggregate" in res and "sage_gemm" in res:
        a, g = res["sage_aggregate"], res["sage_gemm"]
        res["sage_chunk_gather_gemm"] = {
            "kernels": a["kernels"] + g["kernels"],
            "hbm_bytes_per_launch": a["hbm_bytes_per_launch"] + g["hbm_bytes_per_launch"],
            "note": "per row chunk: the gather kernel plus the GEMM kernel that took part of the next "
                    "chunk's gather rows; the GEMM's own A / W / y traffic is included"}
    # the bench configuration these counters belong to (bench JSON of the same command)
    cfg = None
    if len(sys.argv) > 4:
        for line in open(sys.argv[4], errors="replace"):
            if line.startswith("{") and '"metric"' in line:
                j = json.loads(line)
                cfg = j.get("config")
                if tags is TAGS_C4 and cfg is not None:  # forwards in the profiled run: warm-up + timed
                    cfg = dict(cfg, forwards=int(j.get("warmup", 0)) + int(j.get("steps", 0)))
    json.dump({"config": cfg, "kernels": res}, open(out, "w"), indent=1)
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e9, 3) for k, v in res.items()}))


if __name__ == "__main__":
    main()
