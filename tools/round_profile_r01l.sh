set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r01l_prof
timeout -k 10 200 python -u tools/variants.py --variants 0,3 --rounds 7 --reps 10 --dim 64 > gpurun_out/r01l_prof/tail_d64_recheck.log 2>&1 && \
PROF_TAG=r01l_prof bash tools/profile_round.sh
