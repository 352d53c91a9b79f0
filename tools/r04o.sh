#!/bin/bash
# round-4 GPU pass o (run on the box): GPU suite with the small-batch k_gn instance, then
# its A/B against HEAD (asm1) at the per-GPU batches of C2 strong scaling
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04o_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/r04o_gputest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 bash tools/gpu_ab.sh r04o "nlp-filter_amd/mhe/libmhe.so tools/libmhe_asm1.so" "128 256 1024" 4
