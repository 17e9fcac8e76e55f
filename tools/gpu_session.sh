#!/bin/bash
# One GPU session on a gpurun box: the named steps, in order, each under its own time limit;
# the first step that fails ends the call (its status is the call's).  Outputs go to
# gpurun_out/<TAG>_<step>.*.
#
#   bash tools/gpu_session.sh TAG STEP [STEP ...]
#
# steps:
#   box            rocm-smi memory vendor / VBIOS / clocks (never fails the call)
#   tests          the whole -m gpu suite (-x)
#   tests:EXPR     the -m gpu tests selected by -k EXPR
#   testfile:PATH  the -m gpu tests of one file
#   smoke          __graft_entry__.smoke()
#   bench          bench.py, the driver's command (K = 20, W = 5) with the CPU baseline
#   benchq         the same without the CPU baseline
#   config5        bench.py --workload step --L 128 (config 5's per-GPU line)
#   config2        tools/bench_configs.py's config 2 lines (the per-call step at B = 65,536)
#   learner        tools/learner_probe.py (the PPO learner step, fresh and steady state)
#   greedy         tools/bench_greedy.py (AK(3) to 10^6 nodes)
#   bfs            tools/bench_bfs.py 10^7,10^8
#   prof:NAME:ARGS profile_cmd.sh NAME with bench.py arguments ARGS (commas for spaces):
#                  a kernel trace plus separate FETCH_SIZE / WRITE_SIZE passes
#   c2prof         kernel trace and SQ counters of config 2's step (tools/step_pmc.py)
#   script:PATH    any python script of the repo, no arguments
#   py:PATH,ARGS   a python script of the repo with arguments (commas for spaces); output
#                  gpurun_out/TAG_<script name>.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
run_tests() {  # $1 log name, rest: pytest arguments
    local name=$1
    shift
    timeout -k 10 900 python -u -m pytest "$@" -m gpu -q -x --timeout 300 --timeout-method thread \
        -p no:cacheprovider > $OUT/${TAG}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -3 $OUT/${TAG}_${name}.log
    return $rc
}
for step in "$@"; do
    echo "== $step"
    case "$step" in
    box) rocm-smi --showmemvendor --showvbios --showclkfrq --showperflevel > $OUT/${TAG}_box.txt 2>&1 || true ;;
    tests) run_tests gpu_tests tests || exit $? ;;
    tests:*) run_tests gpu_tests_k tests -k "${step#tests:}" || exit $? ;;
    testfile:*) run_tests "gpu_tests_$(basename ${step#testfile:} .py)" "${step#testfile:}" || exit $? ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')" \
            > $OUT/${TAG}_smoke.log 2>&1 || exit 2
        tail -2 $OUT/${TAG}_smoke.log ;;
    bench) timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit 3 ;;
    benchq) timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit 3 ;;
    config5)
        timeout -k 10 400 python -u bench.py --workload step --L 128 --no-cpu --no-bfs --no-search \
            > $OUT/${TAG}_config5.json 2> $OUT/${TAG}_config5.err || exit 4 ;;
    config2) timeout -k 10 300 python -u tools/bench_configs.py > $OUT/${TAG}_config2.json 2> $OUT/${TAG}_config2.err || exit 5 ;;
    learner) timeout -k 10 300 python -u tools/learner_probe.py > $OUT/${TAG}_learner_probe.json 2> $OUT/${TAG}_learner_probe.err || exit 6 ;;
    greedy) timeout -k 10 300 python -u tools/bench_greedy.py > $OUT/${TAG}_greedy.json 2> $OUT/${TAG}_greedy.err || exit 7 ;;
    bfs) timeout -k 10 300 python -u tools/bench_bfs.py 10000000,100000000 > $OUT/${TAG}_bfs.json 2> $OUT/${TAG}_bfs.err || exit 8 ;;
    prof:*)
        spec=${step#prof:}
        name=${spec%%:*}
        args=${spec#*:}
        [ "$args" = "$spec" ] && args=""
        bash profile_cmd.sh ${TAG}_${name} ${args//,/ } || exit 9 ;;
    c2prof)
        (cd /tmp && export TMPDIR=/tmp &&
         timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_c2trace -o c2 --output-format csv \
             -- python3 $R/tools/step_pmc.py --L 36 --B 65536 --K 50 > $OUT/${TAG}_c2trace.log 2>&1 &&
         timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
             SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/${TAG}_c2pmc -o c2 --output-format csv \
             -- python3 $R/tools/step_pmc.py --L 36 --B 65536 --K 50 > $OUT/${TAG}_c2pmc.log 2>&1) || exit 10 ;;
    py:*)
        spec=${step#py:}
        args=${spec//,/ }
        name=$(basename ${args%% *} .py)
        timeout -k 10 300 python -u $args > $OUT/${TAG}_${name}.json 2> $OUT/${TAG}_${name}.err || exit 12 ;;
    script:*)
        s=${step#script:}
        timeout -k 10 300 python -u $s > $OUT/${TAG}_$(basename $s .py).json 2> $OUT/${TAG}_$(basename $s .py).err || exit 11 ;;
    *) echo "unknown step $step"; exit 64 ;;
    esac
done
echo session-done
