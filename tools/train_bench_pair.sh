#!/bin/bash
# The C3 training bench (with the harness legs) and the planted-graph step, each twice on one box.
#   bash tools/train_bench_pair.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1
mkdir -p "$O"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload train --steps 200 --warmup 20 > "$O/c3_$i.log" 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --workload train --graph planted --steps 100 --warmup 10 --no-harness \
    > "$O/planted_$i.log" 2>&1 || exit $?
done
