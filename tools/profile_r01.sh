#!/bin/bash
# rocprofv3 evidence for the bench line: kernel trace + stats, then HBM traffic counters in their
# own passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950). Output under gpurun_out/.
set -euo pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_TAG:-prof_r01}
ARGS=${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc_write.log" 2>&1
echo done > "$OUT/DONE"
