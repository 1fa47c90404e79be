# Same-box A/B of the per-op forward profile: a baseline build of the library (ab/libdie_base.so,
# DIE_LIB_PATH) against the in-tree one, interleaved; each arm autotunes into its own cache.  usage: bash tools/ab_ops.sh <out-name> [rounds] [batch]
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/$1; R=${2:-2}; B=${3:-24}; mkdir -p $O
for r in $(seq 1 $R); do
  DIE_TUNE_CACHE=$PWD/$O/tune_base.json DIE_LIB_PATH=$PWD/ab/libdie_base.so timeout -k 10 300 python3 tools/op_profile.py --arch resnet50 --batch $B \
    --out $O/base_$r > $O/base_$r.txt 2>&1 || exit 1
  DIE_TUNE_CACHE=$PWD/$O/tune_new.json timeout -k 10 300 python3 tools/op_profile.py --arch resnet50 --batch $B --out $O/new_$r > $O/new_$r.txt 2>&1 || exit 1
done
python3 tools/ab_summary.py $O > $O/summary.md
