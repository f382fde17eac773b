# Round check + A/B of the one-launch block-split batch schedule on the C3 training step.
# usage: gpurun -- 'bash tools/ab_blocksplit.sh OUTDIR'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab_blocksplit}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > $O/smoke.log 2>&1 && \
LGCN_BLOCKSPLIT=0 timeout -k 10 300 python -u bench.py --workload train --steps 400 > $O/train_bs0.log 2>&1 && \
LGCN_BLOCKSPLIT=1 timeout -k 10 300 python -u bench.py --workload train --steps 400 > $O/train_bs1.log 2>&1 && \
LGCN_BLOCKSPLIT=0 timeout -k 10 300 python -u bench.py --workload train --steps 400 > $O/train_bs0b.log 2>&1 && \
LGCN_BLOCKSPLIT=1 timeout -k 10 300 python -u bench.py --workload train --steps 400 > $O/train_bs1b.log 2>&1
