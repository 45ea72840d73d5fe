#!/bin/bash
# Round 4 (ran against commit bc54954, reverted after: slower than the general chains kernel): P2P GPU tests, the 16,384-session P2P
# line (the chains form's default range at latency 4) and config 2's P2P shape.
set -u
TAG=${1:-r04t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_p2p.py \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err \
    || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'], r.get('avg_launch_ms'))" gpurun_out/bench_${TAG}_$name.json $name
}
run s16384_1 --workload p2p --sessions 16384
run s16384_2 --workload p2p --sessions 16384
run s16384_canonical --workload p2p --sessions 16384 --p2p-form canonical
run p2pc2 --workload p2p --sessions 4096 --latency 8 --max-prediction 9
echo $TAG done
