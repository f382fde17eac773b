# bench.py (C2 headline, d = 64) with the source-slice size forced (LGCN_SLICE_MB), interleaved
# with the default choice. usage: gpurun -- 'bash tools/ab_slice_mb64.sh OUTTAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab_slice_mb64}; mkdir -p $O
B="timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 100 --warmup 10"
for i in 1 2; do
  $B > $O/d64_default_$i.log 2>&1 || exit 1
  for mb in 6 7 9 10 12 14; do LGCN_SLICE_MB=$mb $B > $O/d64_mb${mb}_$i.log 2>&1 || exit 1; done
done
