#!/bin/bash
# Kernel + memory-copy trace of a training bench, summarised per step (tools/trace_per_step.py,
# marker k_bpr_fused).   bash tools/train_trace.sh TAG [bench args]  (default: the planted C3 step)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1
shift
ARGS=${*:-"--workload train --graph planted --steps 60 --warmup 10 --no-harness"}
mkdir -p "$O"
export TMPDIR=/tmp
D=/tmp/train_trace
rm -rf "$D"
# shellcheck disable=SC2086
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -T -d "$D" -o run --output-format csv -- \
  python3 -u bench.py $ARGS > "$O/bench.log" 2>&1 || exit $?
python3 tools/trace_per_step.py "$D/run_kernel_trace.csv" 40 k_bpr_fused > "$O/per_step.txt" 2>&1 || exit $?
cp "$D"/run_kernel_stats.csv "$O/" ; cp "$D"/run_memory_copy_stats.csv "$O/" 2>/dev/null
python3 - "$D" > "$O/copies.txt" <<'PY' || true
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/*memory_copy_trace.csv"):
    rows = list(csv.DictReader(open(f)))
    print(f, len(rows))
    for r in rows[-20:]:
        print(r)
PY
rm -rf "$D"
