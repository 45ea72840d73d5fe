#!/bin/bash
# Round 4 (experiment, not kept: slower): canonical P2P kernel with each player sin/cos one step ahead: P2P + desync
# GPU tests, the 65,536-session P2P line (three times).
set -u
TAG=${1:-r04u}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_p2p.py \
  tests/test_gpu_desync.py > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload p2p --no-cpu-baseline > gpurun_out/bench_${TAG}_p2p_$i.json 2> gpurun_out/bench_${TAG}_p2p_$i.err \
    || { tail -20 gpurun_out/bench_${TAG}_p2p_$i.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print('p2p', '%.4g' % d['value'], d['ms_per_step'], r.get('avg_launch_ms'))" gpurun_out/bench_${TAG}_p2p_$i.json
done
echo $TAG done
