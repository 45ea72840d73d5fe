#!/bin/bash
# Round 3: branch-engine GPU tests, then config 3 / config 4 bench lines.
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_branch.py tests/test_gpu_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 10; }
tail -1 gpurun_out/pytest_$TAG.log
for W in "--config 3" "--config 3" "--config 4"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline $W "$@" > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/b.json')); r=d.get('roofline') or {}; c=d['config']; print(sys.argv[1], '%.4g'%d['value'], d['ms_per_step'], r.get('avg_kernel_ms_per_round'), c.get('prefix_distinct_frames_per_s'), d.get('parity'))" "$W" | tee -a gpurun_out/summary_$TAG.txt
done
