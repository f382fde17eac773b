#!/bin/bash
# Launch programs (ABI 11): their GPU tests and the training tests that replay captured steps, then
# the C3 / planted training benches with the program (default) and with hipGraph replay.
#   bash tools/program_check.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_program.py tests/test_gpu_training.py tests/test_gpu_harness.py \
  -x -v --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || exit $?
for g in ml25m planted; do
  for i in 1 2; do
    timeout -k 10 300 python -u bench.py --workload train --graph $g --steps 200 --warmup 20 --no-cpu-baseline \
      --tune step_program=1 $([ $g = planted ] && echo --no-harness) > "$O/${g}_program_$i.log" 2>&1 || exit $?
    timeout -k 10 300 python -u bench.py --workload train --graph $g --steps 200 --warmup 20 --no-cpu-baseline \
      --no-harness --tune step_program=0 > "$O/${g}_graph_$i.log" 2>&1 || exit $?
  done
done
