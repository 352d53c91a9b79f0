#!/bin/bash
# A/B variant of libmhe.so for timing runs (van der Pol pairs only, -DMHE_FAST_BUILD):
#   tools/build_ab.sh NAME "-DFLAG=1 ..." [REV "file1 file2 ..."]
# -> ab/libmhe_NAME.so, built from the working tree, or with the listed files taken from
# git revision REV.  Loaded only through MHE_LIB by tools/ab.sh; never by the product.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; VFLAGS=$2; REV=$3; FILES=$4
S=/tmp/mhe_ab_$NAME
rm -rf $S && mkdir -p $S/csrc $S/include $ROOT/ab
cp $ROOT/nlp-filter_amd/csrc/*.h $ROOT/nlp-filter_amd/csrc/*.hip $S/csrc/
cp $ROOT/include/mhe.h $S/include/
for f in $FILES; do git -C $ROOT show $REV:$f > $S/$( [[ $f == include/* ]] && echo include || echo csrc )/$(basename $f); done
FLAGS="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -I$S/include -I$S/csrc -DMHE_FAST_BUILD $VFLAGS"
for s in mhe_gn pair_vdp mhe_ekf mhe_ls; do
  /opt/rocm/bin/hipcc $FLAGS -c -o $S/$s.o $S/csrc/$s.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $ROOT/ab/libmhe_$NAME.so $S/*.o
echo "ab/libmhe_$NAME.so"
