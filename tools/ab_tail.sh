# A/B of the item-pass tail handling (LGCN_SPMM_VARIANT 0 vs 2) at d = 32/64/128/256 on C2 and on
# the C3 training step. usage: gpurun -- 'bash tools/ab_tail.sh OUTDIR'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab_tail}
mkdir -p $O
for d in 32 64 128 256; do
  timeout -k 10 200 python -u tools/variants.py --variants 0,2 --rounds 7 --reps 10 --dim $d > $O/tail_d$d.log 2>&1 || exit 1
done
LGCN_SPMM_VARIANT=0 timeout -k 10 300 python -u bench.py --workload train --steps 400 > $O/train_v0.log 2>&1 && \
LGCN_SPMM_VARIANT=2 timeout -k 10 300 python -u bench.py --workload train --steps 400 > $O/train_v2.log 2>&1
