#!/bin/bash
# Run bench variants on the box: bash tools/gpu_bench.sh <tag> "<args1>" "<args2>" ...
TAG=$1; shift
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
i=0
for a in "$@"; do
  timeout -k 10 300 python -u bench.py $a > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err || { echo "bench '$a' failed"; tail -20 gpurun_out/bench_${TAG}_$i.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$i.json
  i=$((i+1))
done
