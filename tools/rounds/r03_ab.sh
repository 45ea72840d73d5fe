#!/bin/bash
# Round 3: A/B of an experiment library (ggrs_amd/exp/libbase.so, via GGRS_AMD_EXP_LIB) against the
# tree's library on the given bench workload, alternating twice.
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for i in 1 2; do
  for L in base tree; do
    if [ $L = base ]; then export GGRS_AMD_EXP_LIB=$R/ggrs_amd/exp/libbase.so; else unset GGRS_AMD_EXP_LIB; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 11; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/b.json')); r=d.get('roofline') or {}; print(sys.argv[1], '%.4g'%d['value'], d['ms_per_step'], r.get('avg_launch_ms'))" "$L $*" | tee -a gpurun_out/summary_$TAG.txt
  done
done
