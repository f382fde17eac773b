#!/bin/bash
# Planted step: the negatives' grouping on a side stream (tuning grouping_side_stream) vs in line,
# eagerly, as hipGraph replays and as launch programs.   bash tools/side_grouping_probe.sh TAG
# (grouping_side_stream was a tuning field of the measured build only, reverted after this probe:
# DESIGN §10 item 6, profiles/r06zq_side/)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1
mkdir -p "$O"
B="python -u bench.py --workload train --graph planted --steps 100 --warmup 10 --no-harness --no-cpu-baseline"
for i in 1 2; do
  for side in 0 1; do
    timeout -k 10 300 $B --no-graphs --tune grouping_side_stream=$side > "$O/eager_side${side}_$i.log" 2>&1 || exit $?
    timeout -k 10 300 $B --tune step_program=0 --tune grouping_side_stream=$side > "$O/graph_side${side}_$i.log" 2>&1 || exit $?
    timeout -k 10 300 $B --tune grouping_side_stream=$side > "$O/program_side${side}_$i.log" 2>&1 || exit $?
  done
done
