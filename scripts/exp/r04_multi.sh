# Round 4: multi-rank self-launch (host transport on one GPU), C4 on HNSW topology, C5 shard at full size
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_multirank.py tests/test_gpu_hnsw_topology.py > gpurun_out/r04_multirank_pytest.log 2>&1 &&
timeout -k 10 300 python -u bench_hyperbolic.py --gpus 2 --transport host --per-gpu 200000 --queries 2000 --cpu-queries 4 > gpurun_out/r04_hyp_w2.log 2>&1 &&
timeout -k 10 300 python -u bench_gnn.py --gpus 2 --transport host --nodes 200000 --no-cpu > gpurun_out/r04_gnn_w2.log 2>&1 &&
timeout -k 10 300 python -u bench_gnn.py --graph hnsw --nodes 1000000 > gpurun_out/r04_gnn_hnsw1M.log 2>&1 &&
timeout -k 10 600 python -u bench_hyperbolic.py --gpus 1 --per-gpu 6250000 --cpu-queries 4 > gpurun_out/r04_hyp_6p25M.log 2>&1
