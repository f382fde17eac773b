#!/bin/bash
# The C3 and planted training steps with hipGraph replay and eagerly (--no-graphs), one box.
#   bash tools/train_eager_pair.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1
mkdir -p "$O"
for g in ml25m planted; do
  for mode in graphs eager; do
    extra=""; [ $mode = eager ] && extra="--no-graphs"
    timeout -k 10 300 python -u bench.py --workload train --graph $g --steps 200 --warmup 20 --no-harness \
      --no-cpu-baseline $extra > "$O/${g}_${mode}.log" 2>&1 || exit $?
  done
done
