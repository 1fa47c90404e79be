#!/bin/bash
# calibration vs hipBLASLt/MIOpen + counter list + PMC passes on one latency-bound conv
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r18
mkdir -p $O
timeout -k 10 300 python tools/conv_bench.py --batch 16 --ref --json $O/conv_b16.json --md $O/conv_b16.md > $O/b16.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VALU" \
            "TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  n=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/pmc_$n -o p -- python3 tools/conv_one.py --shape s3.3x3 --batch 16 --cfg 7 --splits 1 --iters 20 > $O/pmc_$n.log 2>&1 || { echo "pass $n failed"; exit 1; }
done
echo done
