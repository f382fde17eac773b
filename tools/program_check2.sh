#!/bin/bash
# Launch programs in the multi-rank training modes: the program tests and every exchange test
# (gloo ranks on one GPU, the RCCL branches' code included), eager / graph / program.
#   bash tools/program_check2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_program.py tests/test_gpu_exchange.py tests/test_gpu_dp_recall.py \
  -x -v -s --timeout 600 --timeout-method thread > "$O/tests.log" 2>&1
