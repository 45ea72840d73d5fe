#!/bin/bash
# one extra PMC pass over the default bench: wait / memory-pipe counters of the SyncTest kernel
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/pmc_x -o pmc --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 > $OUT/bench_x.log 2>&1 || exit 12
echo probe done
