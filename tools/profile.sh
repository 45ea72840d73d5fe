#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root): kernel trace + stats, then one
# rocprofv3 pass per PMC group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
# usage: bash tools_profile.sh <tag> [bench args...]
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
BENCH="python3 $R/bench.py --no-cpu-baseline $*"
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- $BENCH > $OUT/bench_trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc --output-format csv -- $BENCH > $OUT/bench_fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc --output-format csv -- $BENCH > $OUT/bench_write.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/pmc_sq -o pmc --output-format csv -- $BENCH > $OUT/bench_sq.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR -d $OUT/pmc_grbm -o pmc --output-format csv -- $BENCH > $OUT/bench_grbm.log 2>&1 || exit 15
echo profile done
