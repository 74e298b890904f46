#!/bin/bash
# Timing-only ablation builds of librvx.so (same sources, one -D each) for scripts/exp/exp_sage_ablate.sh:
#   nonorm  = no normalisation pass; noaggw = the overlapped gather stores no aggregate.
set -e
cd "$(dirname "$0")/.."
make -s ruvector_amd/librvx.so
mkdir -p variants build/var
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Iinclude -Iruvector_amd/csrc -w"
/opt/rocm/bin/hipcc $F -DRVX_AB_NO_NORMALIZE -x hip -c ruvector_amd/csrc/api_graph.cpp -o build/var/api_graph_nonorm.o
/opt/rocm/bin/hipcc $F -DRVX_AB_NO_AGG_WRITE -x hip -c ruvector_amd/csrc/k_aggregate.hip -o build/var/k_aggregate_noaggw.o
L="-shared --offload-arch=gfx950 -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib"
/opt/rocm/bin/hipcc $L -o variants/librvx_nonorm.so $(ls build/*.o | grep -v api_graph.cpp.o) build/var/api_graph_nonorm.o
/opt/rocm/bin/hipcc $L -o variants/librvx_noaggw.so $(ls build/*.o | grep -v k_aggregate.hip.o) build/var/k_aggregate_noaggw.o
/opt/rocm/bin/hipcc $L -o variants/librvx_both.so $(ls build/*.o | grep -v -e k_aggregate.hip.o -e api_graph.cpp.o) build/var/k_aggregate_noaggw.o build/var/api_graph_nonorm.o
