#!/bin/bash
# Round-final evidence at the round's last code (one fresh box): the -m gpu suite, smoke(), the
# driver's bench command, then a kernel trace + stats of that same command (rocprofv3) and the C3
# training bench. usage: gpurun -- 'bash tools/round_final_r06b.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${1:-round_final}
O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > "$O/smoke.log" 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/driver.log" 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d /tmp/prof_final -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$O/prof_bench.log" 2>&1 && \
cp /tmp/prof_final/run_kernel_stats.csv "$O/" && \
timeout -k 10 300 python -u bench.py --workload train --steps 200 --warmup 20 --no-cpu-baseline > "$O/c3_train.log" 2>&1
