# Source-slice size sweep at the narrow widths the 1 x F grids' ranks run (d = 32 / 16 / 8).
# usage: gpurun -- 'bash tools/narrow_slice_sweep.sh OUTTAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-narrow_slices}; mkdir -p $O
timeout -k 10 300 python -u tools/sliced_probe.py --dim 32 --mb 5,8,10,12,14,20 --steps 30 > $O/d32.log 2>&1 && \
timeout -k 10 300 python -u tools/sliced_probe.py --dim 16 --mb 2,3.5,5,7,10 --steps 30 > $O/d16.log 2>&1 && \
timeout -k 10 300 python -u tools/sliced_probe.py --dim 8 --mb 1,1.75,2.5,3.5,5 --steps 30 > $O/d8.log 2>&1
