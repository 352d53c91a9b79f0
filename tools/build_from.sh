#!/bin/bash
# A/B variant of libmhe.so from a copy of the sources with some files taken from a git
# revision: tools/build_from.sh NAME REV "file1 file2 ..." ["-DFLAG ..."]
#   -> ab/libmhe_NAME.so (e.g. the previous revision of one kernel header); never
#   loaded by the product.
set -e
mkdir -p "$(cd "$(dirname "$0")/.." && pwd)/ab"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2; FILES=$3; VFLAGS=$4
S=/tmp/mhe_src_$NAME
rm -rf $S && mkdir -p $S/csrc $S/include
cp $ROOT/nlp-filter_amd/csrc/*.h $ROOT/nlp-filter_amd/csrc/*.hip $S/csrc/
cp $ROOT/include/mhe.h $S/include/
for f in $FILES; do git -C $ROOT show $REV:$f > $S/$( [[ $f == include/* ]] && echo include || echo csrc )/$(basename $f); done
FLAGS="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -I$S/include -I$S/csrc $VFLAGS"
for s in mhe_gn pair_vdp pair_integrators pair_gnss pair_vehicles pair_receivers mhe_ekf mhe_ls; do
  /opt/rocm/bin/hipcc $FLAGS -c -o $S/$s.o $S/csrc/$s.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $ROOT/ab/libmhe_$NAME.so $S/*.o
