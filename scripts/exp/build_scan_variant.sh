#!/bin/bash
# Build variants/librvx_<name>.so: librvx with k_scan.hip compiled under extra macros
# (ablations / experiments; same sources, so the provenance hash still matches).
# usage: scripts/exp/build_scan_variant.sh <name> "-DMACRO ..."
set -eu
cd "$(dirname "$0")/../.."
make -s ruvector_amd/librvx.so
mkdir -p variants build/variants
name=$1; shift
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Iinclude -Iruvector_amd/csrc -Wno-unused-result"
/opt/rocm/bin/hipcc $HIPFLAGS $* -x hip -c ruvector_amd/csrc/k_scan.hip -o build/variants/k_scan_$name.o
objs=$(ls build/*.o | grep -v '/k_scan.hip.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib \
  -o variants/librvx_$name.so $objs build/variants/k_scan_$name.o
echo built variants/librvx_$name.so
