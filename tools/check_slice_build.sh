set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r01m_slicebuild
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_trace.log 2>&1
