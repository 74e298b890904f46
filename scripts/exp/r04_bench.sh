# Round 4: default bench line (N=1), then the same command under rocprofv3 --kernel-trace --stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r04_bench.log 2>&1 &&
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04 -o run -- python3 -u bench.py > gpurun_out/r04_prof_bench.log 2>&1
