#!/bin/bash
# Round 3: request boundary at 4096 sessions: lane groups x host threads.
set -u
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
for a in "--req-groups 2" "--req-groups 4" "--req-groups 2 --req-threads 2" "--req-groups 4 --req-threads 4" "--req-groups 8 --req-threads 8" "--req-groups 8 --req-threads 4"; do
  timeout -k 10 200 python -u bench.py --workload requests --no-cpu-baseline $a > gpurun_out/b.json 2> gpurun_out/b.err || { echo "$a failed"; tail -20 gpurun_out/b.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/b.json')); c=d['config']; print(sys.argv[1], '%.4g'%d['value'], c['us_per_call'], c.get('us_per_call_host_encode_device_handback_session'), d.get('parity'))" "$a" | tee -a gpurun_out/summary_req.txt
done
