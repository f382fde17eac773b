#!/bin/bash
# C5 (HBM stress) profile: bench line with the sampled CPU baseline, kernel trace + stats, and the
# FETCH_SIZE / WRITE_SIZE passes for roofline.traffic (tools/pmc_to_traffic.py <dir> <workload>).
set -euo pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-prof_c5}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python3 -u bench.py --config c5 --steps 5 --warmup 2 > "$OUT/bench_c5.log" 2>&1
P="timeout -k 10 300 rocprofv3"
$P --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/trace.log" 2>&1
$P --pmc FETCH_SIZE -T -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1
$P --pmc WRITE_SIZE -T -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1
echo done > "$OUT/DONE"
