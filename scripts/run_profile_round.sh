set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python bench_hnsw.py --ef 300,400,600 > gpurun_out/hnsw_alone.log 2>&1 || { tail -5 gpurun_out/hnsw_alone.log; exit 1; }
grep -E "build|recall" gpurun_out/hnsw_alone.log | head -8
bash scripts/gpu_profile.sh
