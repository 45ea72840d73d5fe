#!/bin/bash
# Configs 3/4 through the multi-rank exchange path at one rank (RCCL group of one), one all-gather
# per round vs per batch of rounds.  usage: bash tools/xbatch.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
i=0
for a in "--config 4" "--config 4 --exchange-batch 8" "--config 3" "--config 3 --exchange-batch 8"; do
  GGRS_BENCH_DIST=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29600 + i)) bench.py $a --no-cpu-baseline > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err || { tail -20 gpurun_out/bench_${TAG}_$i.err; exit 10; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'])" gpurun_out/bench_${TAG}_$i.json "$a"
  i=$((i+1))
done
echo xbatch done
