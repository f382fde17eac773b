#!/bin/bash
# The clip norm finished inside the update (ABI 11, lgcn_row_adam_reg_fin): the program / training /
# harness GPU tests, then the C3 and planted training benches with it (default) and without
# (norm_in_update_max_rows=0), twice each.
#   bash tools/normfin_check.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_program.py tests/test_gpu_training.py tests/test_gpu_harness.py \
  tests/test_gpu_scatter.py -x -v --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || exit $?
for i in 1 2; do
  for cap in 32768 0; do
    timeout -k 10 300 python -u bench.py --workload train --steps 300 --warmup 30 --no-cpu-baseline \
      --tune norm_in_update_max_rows=$cap $([ $cap = 0 ] && echo --no-harness) > "$O/c3_cap${cap}_$i.log" 2>&1 || exit $?
  done
done
