#!/bin/bash
# Config-2 kernel at other session counts (sessions per GPU; not BASELINE configs: the deployment
# curve) and three repeats of the default bench (run-to-run spread).  usage: bash tools/c2_sweep.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/c2_${TAG}_rep$i.json 2>/dev/null || exit 10
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('repeat', sys.argv[2], '%.4g' % d['value'], d['ms_per_step'])" gpurun_out/c2_${TAG}_rep$i.json $i
done
for L in 1024 2048 8192 16384 65536; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --lanes $L > gpurun_out/c2_${TAG}_l$L.json 2>/dev/null || exit 11
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('sessions', sys.argv[2], '%.4g' % d['value'], d['ms_per_step'])" gpurun_out/c2_${TAG}_l$L.json $L
done
echo c2_sweep done
