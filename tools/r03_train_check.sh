#!/bin/bash
# Training-path changes (grouping scan, no-parking sorted path): the scatter/training GPU tests,
# the C3 and planted training benches, then the per-rank compute probes of the C2 grids
# (reduce mode vs the all_gather mode). usage: bash tools/r03_train_check.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
bash tools/r03_tests.sh $T tests/test_gpu_scatter.py tests/test_gpu_training.py
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload train --steps 200 --warmup 10 > $O/bench_train.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --graph planted --steps 100 --warmup 10 > $O/bench_train_planted.log 2>&1 && \
timeout -k 10 400 python -u tools/reduce_rank_probe.py > $O/reduce_rank_probe.log 2>&1 && \
timeout -k 10 400 python -u tools/shard_rank_probe.py --grids 2x1,4x1,8x1,2x2,4x2,2x4 > $O/shard_rank_probe.log 2>&1
