#!/bin/bash
# Build variants/librvx_<name>.so: librvx with the listed sources compiled under extra macros
# (timing experiments; the provenance hash of the shipped sources is unchanged).
# usage: scripts/exp/build_variant.sh <name> "<macros>" file.hip [file.hip ...]
set -eu
cd "$(dirname "$0")/../.."
make -s ruvector_amd/librvx.so
mkdir -p variants build/variants
name=$1; macros=$2; shift 2
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Iinclude -Iruvector_amd/csrc -Wno-unused-result"
objs=$(ls build/*.o)
for f in "$@"; do
  /opt/rocm/bin/hipcc $HIPFLAGS $macros -x hip -c ruvector_amd/csrc/$f -o build/variants/${f}_$name.o &
  objs=$(echo "$objs" | grep -v "/$f.o$")
done
wait
vobjs=$(for f in "$@"; do echo build/variants/${f}_$name.o; done)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib \
  -o variants/librvx_$name.so $objs $vobjs
echo built variants/librvx_$name.so
