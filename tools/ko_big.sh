#!/bin/bash
# Knock-out builds of the large-system Cholesky (timing probes only; results wrong by design):
#   tools/ko_big.sh <mask> -> tools/libmhe_kob<mask>.so   (MHE_LIB=... python tools/bench_big.py)
set -e
M=$1
C=/root/repo/nlp-filter_amd/csrc
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -I/root/repo/include -I$C -DMHE_BIG_KO=$M \
  -c $C/mhe_gn.hip -o /tmp/kob$M.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o /root/repo/tools/libmhe_kob$M.so /tmp/kob$M.o $C/build/mhe_ekf.o $C/build/mhe_ls.o
