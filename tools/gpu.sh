#!/bin/bash
# One time-limited, logged GPU step on the box (run through gpurun). Replaces round 3's one-shot
# tools/r03_*.sh wrappers.
#
#   bash tools/gpu.sh TAG NAME KIND [ARGS...]      -> gpurun_out/TAG/NAME.log (+ NAME/ for traces)
#
#   KIND pytest ARGS   python -m pytest ARGS -m gpu -v (one process; 300 s per test, 1500 s total)
#   KIND smoke         __graft_entry__.smoke()                                          (120 s)
#   KIND py ARGS       python -u ARGS (bench.py, a tools/ probe, ...)                   (600 s)
#   KIND trace ARGS    rocprofv3 --kernel-trace --stats -d TAG/NAME -- python3 -u ARGS   (600 s)
#   KIND pmc CTRS ARGS rocprofv3 --pmc CTRS (one pass; space-separated counters in one
#                      argument) -d TAG/NAME -- python3 -u ARGS                          (300 s)
#
# Chain steps with && in the gpurun command, so a failing, crashing or timed-out step ends the
# call (exit status is the step's own: 124/137 = time limit, 134 = abort, 139 = fault).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=$1 NAME=$2 KIND=$3
shift 3
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
case "$KIND" in
    pytest)
        timeout -k 10 1500 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread \
            > "$O/$NAME.log" 2>&1 ;;
    smoke)
        timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > "$O/$NAME.log" 2>&1 ;;
    py)
        timeout -k 10 600 python -u "$@" > "$O/$NAME.log" 2>&1 ;;
    trace)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$NAME" -o run -- python3 -u "$@" \
            > "$O/$NAME.log" 2>&1 ;;
    pmc)
        CTRS=$1
        shift
        # shellcheck disable=SC2086  # the counters are one space-separated argument
        timeout -s KILL 300 rocprofv3 --pmc $CTRS -d "$O/$NAME" -o run -- python3 -u "$@" > "$O/$NAME.log" 2>&1 ;;
    *)
        echo "tools/gpu.sh: unknown kind $KIND" >&2
        exit 2 ;;
esac
