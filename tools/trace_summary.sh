#!/bin/bash
# rocprofv3 kernel trace of one command, summarised ON THE BOX (per-step split of a marker
# kernel + the stats CSV) so gpurun_out stays small; the raw trace is deleted.
#   bash tools/trace_summary.sh TAG NAME MARKER STEPS ARGS...   (ARGS: python3 arguments)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=$1 NAME=$2 MARKER=$3 STEPS=$4
shift 4
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
D=/tmp/trace_$NAME
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$D" -o run --output-format csv -- python3 -u "$@" \
    > "$O/$NAME.log" 2>&1 || exit $?
T=$(find "$D" -name '*kernel_trace.csv' | head -1)
S=$(find "$D" -name '*kernel_stats.csv' | head -1)
python3 tools/trace_per_step.py "$T" "$STEPS" "$MARKER" > "$O/$NAME.per_step.txt" 2>&1
cp "$S" "$O/$NAME.kernel_stats.csv"
rm -rf "$D"
