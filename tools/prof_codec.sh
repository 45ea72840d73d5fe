#!/bin/bash
# kernel trace of the codec bench: bash tools/prof_codec.sh <tag>
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $R/bench.py --workload codec --no-cpu-baseline --steps 10 > $OUT/bench_trace.log 2>&1 || exit 11
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/pmc_sq -o pmc --output-format csv -- python3 $R/bench.py --workload codec --no-cpu-baseline --steps 5 > $OUT/bench_sq.log 2>&1 || exit 12
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/pmc_lds -o pmc --output-format csv -- python3 $R/bench.py --workload codec --no-cpu-baseline --steps 5 > $OUT/bench_lds.log 2>&1 || exit 13
head -20 $OUT/trace/trace_kernel_stats.csv
