#!/bin/bash
# Every bench line with its CPU baseline on the GPU box (DESIGN.md §5's table):
# bash tools/all_lines.sh <tag>  ->  gpurun_out/lines_<tag>_<name>.json
TAG=$1
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/lines_${TAG}_$name.json 2> gpurun_out/lines_${TAG}_$name.err || { echo "line $name failed"; tail -20 gpurun_out/lines_${TAG}_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], (d.get('roofline') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/lines_${TAG}_$name.json $name
}
run config3 --config 3
run config4 --config 4
run config5 --config 5
run p2p --workload p2p
run p2p_sparse --workload p2p --sparse
run p2p_c2 --workload p2p --sessions 4096 --latency 8 --max-prediction 9
run p2p_jitter --workload p2p --arrivals jitter
run p2p_stall --workload p2p --arrivals stall
run p2p_jitter4096 --workload p2p --arrivals jitter --sessions 4096 --max-prediction 9
run codec --workload codec
run req --workload requests
run reqp2p --workload requests --req-form p2p --lanes 4096 --req-threads 16 --req-deferred
echo all lines done
