#!/bin/bash
# A/B timing of two builds of the fused kernel on one box (run on the GPU box):
#   tools/ab.sh "<libA.so> <libB.so> ..." [rounds] [batch] [log]   -> gpurun_out/<log> (default ab.log)
# Alternates bench.py --no-cpu runs between the libraries (MHE_LIB).  Kernel shapes are
# build-time choices: build each variant as its own library (tools/build_from.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
LIBS=$1; N=${2:-3}; BATCH=${3:-1024}
O=gpurun_out/${4:-ab.log}
: > $O
for i in $(seq $N); do
  for L in $LIBS; do
    v=$(MHE_LIB=$L timeout -k 10 120 python bench.py --no-cpu --steps 30 --global-batch $BATCH 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
    echo "$L $v" >> $O
  done
done
python - $O <<'PY' >> $O
import collections
r = collections.defaultdict(list)
import sys
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) == 3: r[p[0]].append(float(p[1]))
for k, v in r.items(): print("mean", k, sum(v) / len(v), "n", len(v))
PY
