#!/bin/bash
# In-kernel clock of the split-f16 GEMMs (MI355X_MICROARCH.md DVFS item 6):
# the C4 stack's standalone layer GEMMs at 10M x 768 and the GraphSAGE layer's overlapped GEMM,
# on the diagnostic build variants/librvx_gemmclk.so (gemm_f32.hip with -DRVX_GEMM_CLOCK: every
# gemm_nt_h2w block adds its s_memtime / s_memrealtime deltas, printed per launch; the timings of
# that build are not the product's — each launch is followed by a host wait).
# usage: scripts/exp/build_variant.sh gemmclk -DRVX_GEMM_CLOCK gemm_f32.hip && scripts/exp/gemm_clock.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/gemmclk; mkdir -p $O
RVX_LIB=variants/librvx_gemmclk.so timeout -k 10 300 python bench_gnn.py --nodes ${C4_NODES:-10000000} --steps 1 --warmup 1 --no-cpu > $O/c4.json 2> $O/c4.err || exit 4
RVX_LIB=variants/librvx_gemmclk.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --no-scan --no-c3 --no-c4 --no-c5 --no-hnsw > $O/sage.json 2> $O/sage.err || exit 5
grep "gemm clock" $O/c4.err | awk '{print $3}' | sort | uniq -c | head
python3 - <<'PY'
import re, collections
for f in ("gpurun_out/gemmclk/c4.err", "gpurun_out/gemmclk/sage.err"):
    ghz = collections.defaultdict(list)
    for ln in open(f):
        m = re.search(r"\[gemm clock\] (\S+): ([0-9.]+) GHz \(block-time weighted, ([0-9.]+) block-ms\)", ln)
        if m:
            ghz[m.group(1)].append((float(m.group(2)), float(m.group(3))))
    for tag, v in ghz.items():
        w = sum(b for _, b in v)
        print(f, tag, "launches", len(v), "weighted GHz %.3f" % (sum(g * b for g, b in v) / w), "min %.3f max %.3f" % (min(g for g, _ in v), max(g for g, _ in v)))
PY
