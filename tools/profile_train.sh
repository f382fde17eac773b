# Kernel trace + stats of the C3 training bench (random ML-25M-shaped graph, then the planted graph).
# usage: gpurun -- 'bash tools/profile_train.sh OUTTAG'
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-profile_train}; mkdir -p $O
P="timeout -k 10 300 rocprofv3"
$P --kernel-trace --stats -T -d $O/c3 -o run --output-format csv -- python3 bench.py --workload train --steps 200 --warmup 20 > $O/c3.log 2>&1 && \
$P --kernel-trace --stats -T -d $O/planted -o run --output-format csv -- python3 bench.py --workload train --graph planted --steps 100 --warmup 10 > $O/planted.log 2>&1
