set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$GRAFT_REPO_ROOT/gpurun_out/r10
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for arch in resnet50 vit_b16; do
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/$arch/p1 -o p -- python3 tools/pmc_forward.py $arch 32 2 > $O/$arch.p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/$arch/p2 -o p -- python3 tools/pmc_forward.py $arch 32 2 > $O/$arch.p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/$arch/p3 -o p -- python3 tools/pmc_forward.py $arch 32 2 > $O/$arch.p3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA --output-format csv -d $O/$arch/p4 -o p -- python3 tools/pmc_forward.py $arch 32 2 > $O/$arch.p4.log 2>&1 || exit 1
done
echo "exit=$?"
