cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/r05j_diag.txt
MHE_DIAG_LIB=ab/libmhe_diag_sbW.so timeout -k 10 120 python tools/diag_phases.py 128 4 >> gpurun_out/r05j_diag.txt 2>&1 || exit $?
bash tools/gpu_ab.sh r05j "ab/libmhe_sbA.so ab/libmhe_sbM.so ab/libmhe_sbW.so" "128 256" 3
cat gpurun_out/r05j_diag.txt
