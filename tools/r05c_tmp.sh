cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

B="python bench.py --global-batch 128 --steps 10 --warmup 2 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_r05_sb128 -o run -- $B > gpurun_out/pmc_r05_sb128.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc2_r05_sb128 -o run -- $B > gpurun_out/pmc2_r05_sb128.log 2>&1 || exit $?
ls gpurun_out/pmc_r05_sb128 gpurun_out/pmc2_r05_sb128
