#!/bin/bash
# Persistent split-f16 GEMM tile order in the 10M x 768 GraphSAGE pipeline:
# RVX_GEMM_XSPLIT=0 (each XCD: a row range x all 6 column tiles) vs 1 (an XCD
# pair shares a row range, each XCD 3 column tiles: half the W slice per L2).
# Step time (interleaved x2) and GEMM / gather FETCH_SIZE per launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd); export TMPDIR=/tmp
O=gpurun_out/xsplit; mkdir -p $O
for rep in 1 2; do for v in 0 1; do
  RVX_GEMM_XSPLIT=$v timeout -k 10 300 python3 bench.py --steps 5 --no-cpu --no-hnsw --no-scan > $O/b_${v}_$rep.log 2>&1 || { echo "bench $v failed"; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('$O/b_${v}_$rep.log') if l.startswith('{\"metric')][0]);print('xsplit=$v', round(d['value']/1e9,4), d['kernel_ms'])"
done; done
for v in 0 1; do
  RVX_GEMM_XSPLIT=$v timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$ROOTDIR/$O/pmc_$v" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-hnsw --no-scan > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 - "$O/pmc_$v" $v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: [0.0, 0])
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    key = "gemm_h2g" if "gemm_nt_h2g" in k else ("gather" if "k_aggregate_vec" in k else None)
    if key:
        acc[key][0] += float(r["Counter_Value"]); acc[key][1] += 1
for k, (s, n) in acc.items():
    print("xsplit=%s %s FETCH per launch %.2f GB (x2 corrected, %d launches)" % (sys.argv[2], k, 2 * s * 1024 / n / 1e9, n))
PY
done
