#!/bin/bash
# Round 4 whole-tree pass: GPU tests, smoke, the default bench line, then every workload's bench
# line with its CPU baseline (the DESIGN.md section 5 table), and the RCCL world-1 exchange leg.
set -u
TAG=${1:-r04n}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 11; }
tail -1 gpurun_out/smoke_$TAG.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err \
    || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; c=d.get('cpu_baseline') or {}; print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'], 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'cpu', c.get('value'))" gpurun_out/bench_${TAG}_$name.json $name
}
run c2
run c3 --config 3
run c4 --config 4
run c5 --config 5
run p2p --workload p2p
run p2psparse --workload p2p --sparse
run p2pc2 --workload p2p --sessions 4096 --latency 8 --max-prediction 9
run codec --workload codec
run req --workload requests
run reqp2p --workload requests --req-form p2p --req-groups 2 --req-threads 8 --req-deferred
GGRS_BENCH_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29613 bench.py --no-cpu-baseline \
  > gpurun_out/bench_${TAG}_dist1.json 2> gpurun_out/bench_${TAG}_dist1.err || { tail -20 gpurun_out/bench_${TAG}_dist1.err; exit 13; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('dist1', '%.4g' % d['value'], d.get('exchange'))" gpurun_out/bench_${TAG}_dist1.json
echo $TAG done
