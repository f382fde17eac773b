# bench.py at the 1 x F grids' column widths with the source-slice size forced (LGCN_SLICE_MB),
# interleaved with the default choice (lgcn_amd.plan.slice_bytes_for).
# usage: gpurun -- 'bash tools/ab_slice_mb.sh OUTTAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab_slice_mb}; mkdir -p $O
B="timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 100 --warmup 10"
for i in 1 2; do
  $B --dim 32 > $O/d32_default_$i.log 2>&1 || exit 1
  for mb in 10 12 14; do LGCN_SLICE_MB=$mb $B --dim 32 > $O/d32_mb${mb}_$i.log 2>&1 || exit 1; done
  $B --dim 16 > $O/d16_default_$i.log 2>&1 || exit 1
  for mb in 5 7; do LGCN_SLICE_MB=$mb $B --dim 16 > $O/d16_mb${mb}_$i.log 2>&1 || exit 1; done
done
