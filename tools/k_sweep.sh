#!/bin/bash
# Calls per stage of the chains form (GGRS_SCHED_K) at 4,096 sessions, jitter: bench value and launch ms.
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
for rep in 1 2; do
for k in 8 12 16 20 24; do
  GGRS_SCHED_K=$k timeout -k 10 200 python -u bench.py --workload p2p --arrivals jitter --sessions 4096 --max-prediction 9 --no-cpu-baseline > gpurun_out/ks_$k.json 2>/dev/null || { echo "K $k failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ks_$k.json').read().strip().splitlines()[-1]); print('K $k', d['value'], d['roofline']['avg_launch_ms'], d['parity'].get('every_session_bit_exact'))"
done
done
