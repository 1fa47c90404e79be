cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 tools/decode_bench.py --styles 4dec --batches 32 --iters 3 --packed-only"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/decpmc1 -o run --output-format csv -- $B > gpurun_out/decpmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/decpmc2 -o run --output-format csv -- $B > gpurun_out/decpmc2.log 2>&1
echo rc=$?
