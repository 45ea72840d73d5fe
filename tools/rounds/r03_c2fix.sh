#!/bin/bash
# Round 3: config-2 launch time against frames per launch (the fixed per-launch cost).
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for n in 8 16 32 64 128 256 512; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --frames-per-step $n --steps 50 "$@" > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/b.json')); r=d.get('roofline') or {}; print(sys.argv[1], '%.4g'%d['value'], d['ms_per_step'], r.get('avg_launch_ms'))" $n | tee -a gpurun_out/summary_$TAG.txt
done
