#!/bin/bash
# config 3 (prefix-shared rounds): branch tests, bench, then tools/profile.sh (trace + PMC passes)
# usage: bash tools/r03_prof_c3.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_branch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_branch_$TAG.log 2>&1 || { echo "branch tests failed"; tail -40 gpurun_out/pytest_branch_$TAG.log; exit 10; }
tail -1 gpurun_out/pytest_branch_$TAG.log
timeout -k 10 300 python -u bench.py --config 3 --no-cpu-baseline > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || { tail -20 gpurun_out/bench_c3_$TAG.err; exit 12; }
python -c "import json;d=json.load(open('gpurun_out/bench_c3_$TAG.json'));print('c3', d['value'], d['roofline']['avg_kernel_ms_per_round'], d['parity'])"
bash tools/profile.sh prof_c3_$TAG --config 3 || exit 13
echo prof done
