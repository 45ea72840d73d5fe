#!/bin/bash
# Whole-tree check on the GPU box: GPU tests, smoke, default bench, the plain-launched
# two-rank bench (bench.py spawns its ranks; gloo backend so both share the one GPU), and the
# config-4 two-rank bench with the default batched exchange.
# usage: bash tools/final_check.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 11; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 12; }
cat gpurun_out/bench_$TAG.json
GGRS_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --no-cpu-baseline > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { tail -20 gpurun_out/bench2_$TAG.err; exit 13; }
cat gpurun_out/bench2_$TAG.json
GGRS_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --config 4 --no-cpu-baseline > gpurun_out/bench2c4_$TAG.json 2> gpurun_out/bench2c4_$TAG.err || { tail -20 gpurun_out/bench2c4_$TAG.err; exit 14; }
cat gpurun_out/bench2c4_$TAG.json
echo final_check done
