# Round-end style check on one GPU: the -m gpu suite, the default bench line, smoke().
# usage: gpurun -- 'bash tools/gpu_check.sh OUTDIR'
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > $OUT/smoke.log 2>&1
