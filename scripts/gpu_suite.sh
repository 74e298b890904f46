#!/bin/bash
# GPU test run in two steps: the files named in $FIRST (new / risky kernels) first;
# the rest of the -m gpu suite only if that step neither crashed nor faulted.
# usage: scripts/gpu_suite.sh TAG "tests/a.py tests/b.py"
tag=$1
first=$2
mkdir -p gpurun_out
ign=""
for f in $first; do ign="$ign --ignore=$f"; done
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread $first > gpurun_out/${tag}_a.log 2>&1
rc=$?
if [ $rc -gt 1 ] || grep -qiE "illegal memory|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure" gpurun_out/${tag}_a.log; then
  echo "first step ended with rc=$rc (or a device fault): stopping"; exit 3
fi
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests $ign > gpurun_out/${tag}_b.log 2>&1
rc2=$?
tail -n 3 gpurun_out/${tag}_a.log gpurun_out/${tag}_b.log
exit $(( rc > rc2 ? rc : rc2 ))
