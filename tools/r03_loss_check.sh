#!/bin/bash
# Loss sum folded into the range scatter's launch: scatter + training parity tests, then the train benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03x_loss; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_scatter.py tests/test_gpu_training.py tests/test_gpu_configs.py \
    tests/test_gpu_exchange.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload train --steps 200 --warmup 10 > $O/train_c3_1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload train --steps 200 --warmup 10 > $O/train_c3_2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload train --graph planted --steps 100 --warmup 10 > $O/train_planted.log 2>&1
