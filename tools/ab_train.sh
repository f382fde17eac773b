#!/bin/bash
# Interleaved A/B of the tree's library (new) against a variant .so (old) on the C3 training bench,
# after the listed GPU tests on the tree's build.   bash tools/ab_train.sh TAG VARIANT.so [test files]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1; VAR=$2; shift 2
mkdir -p "$O"
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || exit $?
fi
L=movie-recommender-system-with-gnns_amd/lgcn_amd/liblgcn.so
cp $L "$O/new.so"
B="python -u bench.py --workload train --steps 300 --warmup 30 --no-cpu-baseline --no-harness"
for i in 1 2 3; do
  cp "$O/new.so" $L && timeout -k 10 300 $B > "$O/new_$i.log" 2>&1 || exit 1
  cp "$VAR" $L && timeout -k 10 300 $B > "$O/old_$i.log" 2>&1 || exit 1
done
cp "$O/new.so" $L; rm -f "$O/new.so"
