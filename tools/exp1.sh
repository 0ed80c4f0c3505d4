mkdir -p gpurun_out/exp1
for v in 8 13 14 3; do timeout -k 10 60 python tools/gemm_one.py 16384 4096 4096 0 $v 10 >> gpurun_out/exp1/big.log 2>&1 || exit 1; done
for v in 8 13 14; do timeout -k 10 60 python tools/gemm_one.py 25600 3072 768 1 $v 10 >> gpurun_out/exp1/big.log 2>&1 || exit 1; done
for v in 8 13 14; do timeout -k 10 60 python tools/gemm_one.py 12800 2304 768 0 $v 10 >> gpurun_out/exp1/big.log 2>&1 || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/exp1/pmc_v8 -- python $GRAFT_REPO_ROOT/tools/gemm_one.py 12800 2304 768 0 8 10 > $GRAFT_REPO_ROOT/gpurun_out/exp1/pmc_v8.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/exp1/pmc2_v8 -- python $GRAFT_REPO_ROOT/tools/gemm_one.py 12800 2304 768 0 8 10 > $GRAFT_REPO_ROOT/gpurun_out/exp1/pmc2_v8.log 2>&1 || exit 1
echo done
