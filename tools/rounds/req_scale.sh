#!/bin/bash
# Request boundary at growing session counts, plus the P2P tests and bench.  usage: bash tools/req_scale.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_tests.sh ${TAG}_p2p tests/test_gpu_p2p.py tests/test_gpu_lane_requests.py || exit 10
timeout -k 10 300 python -u bench.py --workload p2p --no-cpu-baseline > gpurun_out/bench_${TAG}_p2p.json 2> gpurun_out/bench_${TAG}_p2p.err || exit 11
cat gpurun_out/bench_${TAG}_p2p.json
for L in 4096 16384 32768 65536; do
  timeout -k 10 300 python -u bench.py --workload requests --lanes $L --no-cpu-baseline > gpurun_out/bench_${TAG}_$L.json 2> gpurun_out/bench_${TAG}_$L.err || { tail -20 gpurun_out/bench_${TAG}_$L.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['us_per_call'])" gpurun_out/bench_${TAG}_$L.json $L
done
echo req_scale done
