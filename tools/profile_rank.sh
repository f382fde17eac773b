# rocprofv3 kernel trace of one rank's reduce-mode C2 step at 4x2 (tools/reduce_rank_probe.py,
# overlapped and fused orders) and the one-GPU d=32 full-graph step for comparison.
# usage: gpurun -- 'bash tools/profile_rank.sh OUTTAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rank_prof}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/reduce_rank_probe.py --grids 4x2 --orders overlapped,fused,overlapped+g,fused+g > $O/probe.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 tools/reduce_rank_probe.py --grids 4x2 --orders overlapped+g --steps 20 > $O/trace.log 2>&1
