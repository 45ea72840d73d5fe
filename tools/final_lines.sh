#!/bin/bash
# The whole-tree check, then the P2P lines the last kernel changes touch (fixed latency, config 2's
# P2P shape, jitter, stall, jitter 4,096), each with its CPU baseline.
#   bash tools/final_lines.sh <tag>
set -e
TAG=$1
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out/$TAG
bash tools/final_check.sh $TAG
for a in "p2p:--workload p2p" "p2p_c2:--workload p2p --sessions 4096 --latency 8 --max-prediction 9" "p2p_jitter:--workload p2p --arrivals jitter" "p2p_stall:--workload p2p --arrivals stall" "p2p_jitter4096:--workload p2p --arrivals jitter --sessions 4096 --max-prediction 9"; do
  name=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python -u bench.py $args > gpurun_out/$TAG/lines_${TAG}_$name.json 2> gpurun_out/$TAG/$name.err
  echo "$name done"
done
