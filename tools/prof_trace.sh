#!/bin/bash
# kernel trace of one bench configuration: bash tools/prof_trace.sh <tag> [bench args...]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_trace.log 2>&1 || exit 11
cut -c1-200 $OUT/trace/trace_kernel_stats.csv | head -8
