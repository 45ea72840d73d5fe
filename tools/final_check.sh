#!/bin/bash
# Whole-tree check on the GPU box: every GPU test, smoke(), the default bench, and a two-rank
# rehearsal of the multi-process bench path on this one GPU (gloo backend, both ranks on cuda:0).
# usage: bash tools/final_check.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 11; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 12; }
cat gpurun_out/bench_$TAG.json
GGRS_BENCH_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { tail -20 gpurun_out/bench2_$TAG.err; exit 13; }
cat gpurun_out/bench2_$TAG.json
echo final_check done
