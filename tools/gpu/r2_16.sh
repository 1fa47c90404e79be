#!/bin/bash
# Fresh PMC passes on the production (autotuned, v5) kernels at B=32 and B=16, fp32; ViT-B/16 fp32 bench.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_16
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd /tmp && export TMPDIR=/tmp
cd $R
for B in 32 16; do
  timeout -k 10 300 python3 tools/pmc_forward.py resnet50 $B 1 fp32 tuned > $O/tune_$B.log 2>&1 || { tail $O/tune_$B.log; exit 1; }
  D=$O/fp32_b$B
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $D/p1 -o p -- python3 tools/pmc_forward.py resnet50 $B 2 fp32 tuned > $D.p1.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $D/p2 -o p -- python3 tools/pmc_forward.py resnet50 $B 2 fp32 tuned > $D.p2.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $D/p3 -o p -- python3 tools/pmc_forward.py resnet50 $B 2 fp32 tuned > $D.p3.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA --output-format csv -d $D/p4 -o p -- python3 tools/pmc_forward.py resnet50 $B 2 fp32 tuned > $D.p4.log 2>&1 || { tail $D.p*.log; exit 1; }
  python3 tools/pmc_summary.py $D --title "resnet50 fp32 B=$B tuned (1-stage LDS-DMA variant, fused stem)" --note "production (autotuned) kernel configs, eager launches" > $O/pmc_fp32_b$B.md || exit 1
  tail -1 $O/pmc_fp32_b$B.md
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --arch vit_b16 > $O/vit_fp32.json 2> $O/vit_fp32.err || { tail -20 $O/vit_fp32.err; exit 1; }
python -c "import json;d=json.load(open('$O/vit_fp32.json'));print('vit fp32',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('device_ms_per_batch'),d.get('direct_worker',{}).get('rps_this_rank'))"
