#!/bin/bash
# Round 3: config-2 kernel check: SyncTest GPU tests, then the default bench three times.
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sincosf.py tests/test_gpu_synctest.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -1 gpurun_out/pytest_$TAG.log
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/b.json')); r=d.get('roofline') or {}; print('%.4g'%d['value'], d['ms_per_step'], r.get('avg_launch_ms', r.get('avg_kernel_ms_per_round')), d.get('parity'))" | tee -a gpurun_out/summary_$TAG.txt
done
