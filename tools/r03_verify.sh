#!/bin/bash
# After removing the memset node from lgcn_group_keys: the planted training bench (captured steps,
# counting-sort grouping) first, then the affected GPU tests and the bench lines; stops at the first
# crash. usage: bash tools/r03_verify.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u bench.py --workload train --graph planted --steps 100 --warmup 10 > $O/bench_train_planted.log 2>&1 || exit $?
bash tools/r03_tests.sh $T tests/test_gpu_scatter.py tests/test_gpu_training.py tests/test_gpu_exchange.py tests/test_gpu_configs.py
rc=$?
[ $rc -le 1 ] || exit $rc
bash tools/r03_benches.sh $T
