# -m gpu suite + the C3 training bench (twice; PLANTED=1: and the planted graph's once). usage: gpurun -- 'bash tools/check_train.sh OUTDIR'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-check_train}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --steps 400 > $O/train_a.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --steps 400 > $O/train_b.log 2>&1 || exit 1
if [ -n "$PLANTED" ]; then
  timeout -k 10 300 python -u bench.py --workload train --graph planted --steps 150 --warmup 10 > $O/planted.log 2>&1 || exit 1
fi
