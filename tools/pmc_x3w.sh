set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_x3w
cd /tmp
export GEMM_AB_CASES="enc0 fwd" GEMM_AB_KERNELS=wide
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d $R/gpurun_out/pmc_x3w/p1 -o p1 -f csv -- python3 $R/tools/gemm_ab.py 5 > $R/gpurun_out/pmc_x3w/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_x3w/p2 -o p2 -f csv -- python3 $R/tools/gemm_ab.py 5 > $R/gpurun_out/pmc_x3w/p2.log 2>&1 || exit 1
