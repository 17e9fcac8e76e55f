set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_rollout.py abv/libacx_prewait.so abv/libacx_base.so abv/libacx_nt0.so abv/libacx_occ4.so abv/libacx_occ6.so --reps 7 > gpurun_out/ab1.json 2> gpurun_out/ab1.err
