cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab.sh r05_sb "ab/libmhe_nosb.so ab/libmhe_head.so" "128 256 512 1024" 3 || exit 1
