#!/bin/bash
# Round 4 experiment: config 3 with the prefix kernel's ring saves write-through (sc1,
# GGRS_EXP_WT=1) against the default policy, A/B twice on one box.
set -u
TAG=${1:-r04h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for i in 1 2; do
  for wt in 0 1; do
    if [ $wt = 1 ]; then export GGRS_EXP_WT=1; else unset GGRS_EXP_WT; fi
    timeout -k 10 200 python -u bench.py --config 3 --no-cpu-baseline > gpurun_out/bench_${TAG}_c3_wt${wt}_$i.json \
      2> gpurun_out/bench_${TAG}_c3_wt${wt}_$i.err || { tail -20 gpurun_out/bench_${TAG}_c3_wt${wt}_$i.err; exit 11; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c3 wt', sys.argv[2], '%.4g' % d['value'], d['ms_per_step'])" gpurun_out/bench_${TAG}_c3_wt${wt}_$i.json $wt
  done
done
unset GGRS_EXP_WT
echo $TAG done
