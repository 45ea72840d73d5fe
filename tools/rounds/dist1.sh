#!/bin/bash
# Every bench workload through the multi-rank code path at one rank (RCCL group of one, launched
# as the driver launches N ranks): rank 0's stdout must be exactly one JSON line.
# usage: bash tools/dist1.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
i=0
for a in "" "--config 5 --steps 3" "--workload p2p" "--workload codec" "--workload requests"; do
  GGRS_BENCH_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29700 + i)) bench.py $a --gpus 1 --no-cpu-baseline > gpurun_out/dist1_${TAG}_$i.json 2> gpurun_out/dist1_${TAG}_$i.err || { tail -20 gpurun_out/dist1_${TAG}_$i.err; exit 10; }
  n=$(wc -l < gpurun_out/dist1_${TAG}_$i.json)
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], 'lines', '%.4g' % d['value'], d['ms_per_step'])" gpurun_out/dist1_${TAG}_$i.json "[$a]" "$n"
  i=$((i+1))
done
echo dist1 done
