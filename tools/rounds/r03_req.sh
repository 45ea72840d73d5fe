#!/bin/bash
# request boundary: lane-request GPU tests, the requests bench in its forms.  usage: bash tools/r03_req.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lane_requests.py tests/test_gpu_requests.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_req_$TAG.log 2>&1 || { echo "request tests failed"; tail -50 gpurun_out/pytest_req_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_req_$TAG.log
for spec in "g1:--req-groups 1" "g2:--req-groups 2" "g4:--req-groups 4" "p2p2:--req-form p2p --req-groups 2" "p2p1:--req-form p2p --req-groups 1"; do
  name=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python -u bench.py --workload requests --no-cpu-baseline $a > gpurun_out/req_${TAG}_$name.json 2> gpurun_out/req_${TAG}_$name.err || { tail -20 gpurun_out/req_${TAG}_$name.err; exit 11; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['us_per_call'], d['config'].get('us_per_call_host_encode_device_handback_session'), d['parity'])" gpurun_out/req_${TAG}_$name.json $name
done
echo req done
