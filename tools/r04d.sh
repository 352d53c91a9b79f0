#!/bin/bash
# round-4 GPU pass d (run on the box): suite + bench + k_gn hoist A/B, then the large-path
# A/Bs (assemble: LDS-staged vs coalesced vs round-3; chol: 8-wide K4 slab)
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_quick.sh r04d "nlp-filter_amd/mhe/libmhe.so tools/libmhe_nohoist.so" "1024 256" || exit $?
timeout -k 10 500 bash tools/ab_big_env.sh "C3:1024" "nlp-filter_amd/mhe/libmhe.so tools/libmhe_asmcoal.so tools/libmhe_asm03.so tools/libmhe_k4.so" 2 || exit $?
cp gpurun_out/ab_big_env.log gpurun_out/r04d_ab_big_C3.txt
timeout -k 10 300 bash tools/ab_big_env.sh "C4:256" "nlp-filter_amd/mhe/libmhe.so tools/libmhe_asmcoal.so" 2 || exit $?
cp gpurun_out/ab_big_env.log gpurun_out/r04d_ab_big_C4.txt
