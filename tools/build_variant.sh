#!/bin/bash
# Full A/B variant of libmhe.so (all plug-in pairs): tools/build_variant.sh NAME "-DFLAG=1 ..."
# -> ab/libmhe_NAME.so (objects in /tmp/mhe_variant_NAME); never loaded by the product.
set -e
mkdir -p "$(cd "$(dirname "$0")/.." && pwd)/ab"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; VFLAGS=$2
B=/tmp/mhe_variant_$NAME
mkdir -p $B
FLAGS="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -I$ROOT/include -I$ROOT/nlp-filter_amd/csrc $VFLAGS"
for s in mhe_gn pair_vdp pair_integrators pair_gnss pair_vehicles pair_receivers mhe_ekf mhe_ls; do
  /opt/rocm/bin/hipcc $FLAGS -c -o $B/$s.o $ROOT/nlp-filter_amd/csrc/$s.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $ROOT/ab/libmhe_$NAME.so $B/*.o
