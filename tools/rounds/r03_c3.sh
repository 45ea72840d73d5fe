#!/bin/bash
# config-3 prefix-shared rounds: branch GPU tests, the config-3 bench, and its kernel trace
# usage: bash tools/r03_c3.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_branch.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_branch_$TAG.log 2>&1 || { echo "branch tests failed"; tail -40 gpurun_out/pytest_branch_$TAG.log; exit 10; }
tail -3 gpurun_out/pytest_branch_$TAG.log
timeout -k 10 300 python -u bench.py --config 3 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || { tail -20 gpurun_out/bench_c3_$TAG.err; exit 12; }
cat gpurun_out/bench_c3_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_$TAG -o trace -- python -u bench.py --config 3 --no-cpu-baseline > gpurun_out/prof_c3_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_c3_$TAG.log; exit 13; }
find gpurun_out/prof_c3_$TAG -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -8
echo c3 done
