#!/bin/bash
# The bench lines of a round check, each under its own time limit, stopping at the first failure.
# usage: bash tools/r03_benches.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > $O/bench_gpus2_gloo.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --steps 200 --warmup 10 > $O/bench_train.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --graph planted --steps 100 --warmup 10 > $O/bench_train_planted.log 2>&1
