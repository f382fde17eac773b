#!/bin/bash
# Column-sharded training with the segmented graph capture: its bitwise test against the eager
# step, then the train bench per mode: one GPU, and 2 / 4 gloo ranks on the one GPU (path and
# per-step cost only: the ranks share the card and gloo goes through host memory).
# usage: gpurun -- 'bash tools/r03_cols.sh TAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03_cols}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_exchange.py -k "column_sharded or world1 or dp2" -x -v --timeout 300 --timeout-method thread > $O/pytest_cols.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --no-cpu-baseline > $O/train_1gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --gpus 2 --dist-backend gloo --dp-mode columns --steps 40 --warmup 40 --no-cpu-baseline > $O/train_cols2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --gpus 2 --dist-backend gloo --dp-mode columns --no-graphs --steps 40 --warmup 40 --no-cpu-baseline > $O/train_cols2_eager.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --gpus 4 --dist-backend gloo --dp-mode columns --steps 40 --warmup 40 --no-cpu-baseline > $O/train_cols4.log 2>&1
