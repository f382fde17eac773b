#!/bin/bash
# Row Adam early last[row] A/B: the training parity tests on the default build (last[row] loaded
# beside the claim), then the C3 train bench interleaved default / late-load variant (tools/ab_lib.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03x_early; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_configs.py tests/test_gpu_exchange.py -x -q \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
bash tools/ab_lib.sh r03x_early/ab_c3 ab/adam_late.so --workload train --steps 200 --warmup 10 && \
bash tools/ab_lib.sh r03x_early/ab_planted ab/adam_late.so --workload train --graph planted --steps 100 --warmup 10
