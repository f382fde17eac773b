#!/bin/bash
# Memory-side traffic per training-step kernel (planted C3 step): FETCH_SIZE and WRITE_SIZE in
# their own --pmc passes plus a kernel trace for the durations, summarised on the box by
# tools/train_pmc_summary.py (the raw CSVs are deleted).   bash tools/train_pmc.sh TAG [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=$1
shift
ARGS=${*:-"--workload train --graph planted --steps 12 --warmup 3 --no-harness"}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
D=/tmp/train_pmc
rm -rf "$D"
# shellcheck disable=SC2086
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$D/trace" -o run --output-format csv -- python3 -u bench.py $ARGS > "$O/trace.log" 2>&1 || exit $?
# shellcheck disable=SC2086
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE -T -d "$D/fetch" -o run --output-format csv -- python3 -u bench.py $ARGS > "$O/fetch.log" 2>&1 || exit $?
# shellcheck disable=SC2086
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE -T -d "$D/write" -o run --output-format csv -- python3 -u bench.py $ARGS > "$O/write.log" 2>&1 || exit $?
python3 tools/train_pmc_summary.py "$D" > "$O/summary.txt" 2>&1 || exit $?
rm -rf "$D"
