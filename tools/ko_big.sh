#!/bin/bash
# Knock-out builds of the large-system Cholesky (timing probes only; results wrong by design,
# X frozen so every iteration solves the same system):
#   tools/ko_big.sh <mask> -> tools/libmhe_kob<mask>.so   (MHE_LIB=... python tools/bench_big.py)
# mask bits: mhe_big.h MHE_BIG_KO; 64 = nothing knocked out (the baseline with X frozen)
set -e
bash "$(dirname "$0")/build_variant.sh" kob$1 "-DMHE_BIG_KO=$1"
