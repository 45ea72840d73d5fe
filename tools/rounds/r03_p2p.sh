#!/bin/bash
# Round 3: P2P / branch / particle GPU tests, then P2P, sparse P2P, config 4, config 3 and config 5 bench lines.
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_desync.py tests/test_gpu_branch.py tests/test_gpu_exchange.py tests/test_gpu_particles.py tests/test_gpu_requests.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 10; }
tail -1 gpurun_out/pytest_$TAG.log
for W in "--workload p2p" "--workload p2p --sparse" "--config 4" "--config 3"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline $W > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/b.json')); r=d.get('roofline') or {}; print(sys.argv[1], '%.4g'%d['value'], d['ms_per_step'], r.get('avg_launch_ms', r.get('avg_kernel_ms_per_round')), d.get('parity'))" "$W" | tee -a gpurun_out/summary_$TAG.txt
done
