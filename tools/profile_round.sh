#!/bin/bash
# Round profile: kernel trace + stats of the default bench, then HBM-traffic counters in their own
# passes (FETCH_SIZE / WRITE_SIZE), for the bench and for the FETCH_SIZE calibration run.
set -euo pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_TAG:-prof_round}
mkdir -p "$OUT"
cd "$R"
P="timeout -k 10 300 rocprofv3"
$P --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- python3 bench.py > "$OUT/trace.log" 2>&1
$P --pmc FETCH_SIZE -T -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1
$P --pmc WRITE_SIZE -T -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1
$P --pmc FETCH_SIZE -T -d "$OUT/calib_fetch" -o run --output-format csv -- python3 tools/calib_fetch.py > "$OUT/calib_fetch.log" 2>&1
$P --pmc WRITE_SIZE -T -d "$OUT/calib_write" -o run --output-format csv -- python3 tools/calib_fetch.py > "$OUT/calib_write.log" 2>&1
echo done > "$OUT/DONE"
