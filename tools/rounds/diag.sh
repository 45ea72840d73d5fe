#!/bin/bash
# Counter diagnosis of one bench configuration (run on the GPU box from the repo root):
# two rocprofv3 --pmc passes of SQ issue/wait counters.  usage: bash tools/diag.sh <tag> [bench args...]
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
BENCH="python3 $R/bench.py --no-cpu-baseline --steps 5 $*"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/pmc_a -o pmc --output-format csv -- $BENCH > $OUT/a.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/pmc_b -o pmc --output-format csv -- $BENCH > $OUT/b.log 2>&1 || exit 12
echo diag done
