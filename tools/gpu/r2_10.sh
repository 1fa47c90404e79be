#!/bin/bash
# PMC passes over the tuned (production-config) fp32 and bf16 ResNet50 forward at B=32, plus the
# DP world=1 bench after enabling pacing under DP.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_10
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mode dp > $O/dp1.json 2> $O/dp1.err || { tail -20 $O/dp1.err; exit 1; }
python -c "import json;d=json.load(open('$O/dp1.json'));print('dp1',round(d['value']),d['p50_ms'],d.get('dp_batches_rank0'),d.get('device_ms_per_batch'))"
for prec in fp32 bf16; do
  # warm the tune cache without the profiler
  timeout -k 10 300 python3 tools/pmc_forward.py resnet50 32 1 $prec tuned > $O/tune_$prec.log 2>&1 || { tail $O/tune_$prec.log; exit 1; }
  D=$O/$prec
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $D/p1 -o p -- python3 tools/pmc_forward.py resnet50 32 2 $prec tuned > $D.p1.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $D/p2 -o p -- python3 tools/pmc_forward.py resnet50 32 2 $prec tuned > $D.p2.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $D/p3 -o p -- python3 tools/pmc_forward.py resnet50 32 2 $prec tuned > $D.p3.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA --output-format csv -d $D/p4 -o p -- python3 tools/pmc_forward.py resnet50 32 2 $prec tuned > $D.p4.log 2>&1 || { tail $D.p*.log; exit 1; }
  python3 tools/pmc_summary.py $D --title "resnet50 $prec B=32 tuned" --note "production (autotuned) kernel configs, eager launches" > $O/pmc_$prec.md || exit 1
  tail -3 $O/pmc_$prec.md
done
