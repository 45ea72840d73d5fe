#!/bin/bash
# Request-boundary iteration on the GPU box: lane-request parity tests, the requests bench at 4096
# and 16,384 sessions, the per-call breakdown (tools/req_diag.py).  usage: bash tools/req_round.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_tests.sh ${TAG}_req tests/test_gpu_lane_requests.py tests/test_gpu_requests.py || exit 10
for L in 4096 16384; do
  timeout -k 10 300 python -u bench.py --workload requests --lanes $L --no-cpu-baseline > gpurun_out/bench_${TAG}_$L.json 2> gpurun_out/bench_${TAG}_$L.err || { tail -20 gpurun_out/bench_${TAG}_$L.err; exit 11; }
  cat gpurun_out/bench_${TAG}_$L.json
done
timeout -k 10 300 python -u tools/req_diag.py 4096 1 > gpurun_out/req_diag_$TAG.json 2>&1 || exit 12
cat gpurun_out/req_diag_$TAG.json
echo req_round done
