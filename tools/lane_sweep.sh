#!/bin/bash
# Config-2 kernel time versus sessions per GPU (waves per SIMD): bash tools/lane_sweep.sh <tag> [lanes...]
TAG=$1; shift
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
for l in "$@"; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --lanes $l --steps 10 > gpurun_out/sweep_${TAG}_$l.json 2> gpurun_out/sweep_${TAG}_$l.err || { echo "lanes $l failed"; tail -5 gpurun_out/sweep_${TAG}_$l.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_${TAG}_$l.json').read().strip().splitlines()[-1]); print($l, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'] if 'avg_launch_ms' in d['roofline'] else '')"
done
