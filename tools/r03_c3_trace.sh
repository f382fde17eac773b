#!/bin/bash
# C3 training step kernel trace: per-step kernel times (tools/trace_per_step.py), trace kept in /tmp.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03x_c3trace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d /tmp/c3trace -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --workload train --steps 60 --warmup 10 > $O/bench_train.log 2>&1 && \
cp /tmp/c3trace/run_kernel_stats.csv $O/ && \
python3 tools/trace_per_step.py /tmp/c3trace/run_kernel_trace.csv 50 distribution_elementwise > $O/per_step.txt 2>&1
