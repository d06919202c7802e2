#!/bin/bash
# Build an experimental variant of libddr_mc.so with extra preprocessor flags.
# Usage: bash tools/build_variant.sh NAME "-DDDR_CHUNK=8 ..."   -> ddr_amd/lib/libddr_mc_NAME.so
set -e
NAME=$1; shift
R=$(cd $(dirname $0)/.. && pwd)
OBJ=/tmp/ddr_variant_$NAME
mkdir -p $OBJ
cd $R/ddr_amd/csrc
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function $*"
rm -f $OBJ/*.o
for s in graph.cpp collate.cpp capi.cpp route.hip trisolve.hip geometry.hip devgraph.hip pnet.hip train.hip; do
  /opt/rocm/bin/hipcc $FL -x hip -c $s -o $OBJ/$s.o &
done
wait
for s in graph.cpp collate.cpp capi.cpp route.hip trisolve.hip geometry.hip devgraph.hip pnet.hip train.hip; do [ -f $OBJ/$s.o ] || { echo "variant build failed: $s"; exit 1; }; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $R/ddr_amd/lib/libddr_mc_$NAME.so $OBJ/*.o
echo built $R/ddr_amd/lib/libddr_mc_$NAME.so
