#!/bin/bash
# Round 4 first check: the null-stream exchange test, config-2 P2P parity, the ABI test, then the
# config-2 P2P bench line, the gloo 2-rank bench with its exchange key and the one-rank RCCL one.
set -u
TAG=${1:-r04a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_exchange.py tests/test_abi.py tests/test_gpu_p2p.py tests/test_gpu_branch.py tests/test_gpu_lane_requests.py \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u bench.py --workload p2p --sessions 4096 --latency 8 --max-prediction 9 \
  > gpurun_out/bench_${TAG}_p2pc2.json 2> gpurun_out/bench_${TAG}_p2pc2.err || { tail -20 gpurun_out/bench_${TAG}_p2pc2.err; exit 11; }
cat gpurun_out/bench_${TAG}_p2pc2.json
timeout -k 10 300 python -u bench.py --workload p2p --sessions 4096 --latency 8 --max-prediction 9 --p2p-form flat --no-cpu-baseline \
  > gpurun_out/bench_${TAG}_p2pc2flat.json 2> gpurun_out/bench_${TAG}_p2pc2flat.err || { tail -20 gpurun_out/bench_${TAG}_p2pc2flat.err; exit 11; }
cat gpurun_out/bench_${TAG}_p2pc2flat.json
for S in 16384 65536; do
for F in chains canonical flat_queues; do
timeout -k 10 300 python -u bench.py --workload p2p --sessions $S --p2p-form $F --no-cpu-baseline \
  > gpurun_out/bench_${TAG}_p2p${F}$S.json 2> gpurun_out/bench_${TAG}_p2p${F}$S.err || { tail -20 gpurun_out/bench_${TAG}_p2p${F}$S.err; exit 11; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], d['roofline']['avg_launch_ms'])" gpurun_out/bench_${TAG}_p2p${F}$S.json $F$S
done
done
timeout -k 10 300 python -u bench.py --workload p2p --sparse --no-cpu-baseline > gpurun_out/bench_${TAG}_p2psparse.json 2> gpurun_out/bench_${TAG}_p2psparse.err || { tail -20 gpurun_out/bench_${TAG}_p2psparse.err; exit 11; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('sparse', '%.4g' % d['value'], d['roofline']['avg_launch_ms'])" gpurun_out/bench_${TAG}_p2psparse.json
GGRS_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 \
  > gpurun_out/bench_${TAG}_gloo2.json 2> gpurun_out/bench_${TAG}_gloo2.err || { tail -20 gpurun_out/bench_${TAG}_gloo2.err; exit 12; }
cat gpurun_out/bench_${TAG}_gloo2.json
GGRS_BENCH_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --no-cpu-baseline \
  > gpurun_out/bench_${TAG}_dist1.json 2> gpurun_out/bench_${TAG}_dist1.err || { tail -20 gpurun_out/bench_${TAG}_dist1.err; exit 13; }
cat gpurun_out/bench_${TAG}_dist1.json
i=0
for a in "--req-groups 1" "--req-groups 1 --req-deferred" "--req-groups 1 --session-us 20" "--req-groups 1 --session-us 20 --req-deferred" "--req-groups 2 --req-threads 8 --req-deferred" "--req-groups 1 --req-threads 8 --req-deferred --session-us 20"; do
  timeout -k 10 200 python -u bench.py --workload requests --req-form p2p --no-cpu-baseline $a \
    > gpurun_out/bench_${TAG}_req$i.json 2> gpurun_out/bench_${TAG}_req$i.err || { tail -20 gpurun_out/bench_${TAG}_req$i.err; exit 14; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], '%.4g' % d['value'], c['us_per_call'], c.get('us_per_call_host_encode_device_handback_session'))" gpurun_out/bench_${TAG}_req$i.json "$a"
  i=$((i+1))
done
echo r04a done
