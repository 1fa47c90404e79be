#!/bin/bash
# Per-op fp32 time vs batch (fixed per-batch cost), B=16 PMC pass.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_17
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd /tmp && export TMPDIR=/tmp
cd $R
for B in 8 16 24; do
  timeout -k 10 300 python -u tools/op_profile.py --arch resnet50 --batch $B --precision fp32 --out $O/ops_fp32_b$B.md > $O/ops_$B.log 2>&1 || { tail -20 $O/ops_$B.log; exit 1; }
  sed -n 3p $O/ops_fp32_b$B.md.md
done
B=16
D=$O/fp32_b$B
timeout -k 10 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $D/p1 -o p -- python3 tools/pmc_forward.py resnet50 $B 2 fp32 tuned > $D.p1.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $D/p2 -o p -- python3 tools/pmc_forward.py resnet50 $B 2 fp32 tuned > $D.p2.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $D/p3 -o p -- python3 tools/pmc_forward.py resnet50 $B 2 fp32 tuned > $D.p3.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA --output-format csv -d $D/p4 -o p -- python3 tools/pmc_forward.py resnet50 $B 2 fp32 tuned > $D.p4.log 2>&1 || { tail $D.p*.log; exit 1; }
python3 tools/pmc_summary.py $D --title "resnet50 fp32 B=16 tuned" --note "production (autotuned) kernel configs, eager launches" > $O/pmc_fp32_b16.md || exit 1
tail -1 $O/pmc_fp32_b16.md
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --arch vit_b16 > $O/vit_fp32.json 2> $O/vit_fp32.err || { tail -20 $O/vit_fp32.err; exit 1; }
python -c "import json;d=json.load(open('$O/vit_fp32.json'));print('vit fp32',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('device_ms_per_batch'),d.get('direct_worker',{}).get('rps_this_rank'))"
