#!/bin/bash
# One GPU-box pass: GPU parity tests, default bench, kernel-trace + PMC profile of the default bench.
# usage: bash tools/round.sh <tag> [extra bench command...]
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 10; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 11; }
cat gpurun_out/bench_$TAG.json
if [ $# -gt 0 ]; then
  timeout -k 10 300 "$@" > gpurun_out/extra_$TAG.log 2>&1 || { echo "extra failed"; tail -20 gpurun_out/extra_$TAG.log; exit 12; }
  cat gpurun_out/extra_$TAG.log
fi
bash tools/profile.sh $TAG --steps 10 || exit 13
echo round done
