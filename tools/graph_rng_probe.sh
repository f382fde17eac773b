set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/graph_rng; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 tools/graph_rng_probe.py > $O/log.txt 2>&1
