#!/bin/bash
# PMC passes over config 2 at several session counts (waves per SIMD): bash tools/pmc_probe.sh <tag> "<lanes...>" [lib]
set -u
TAG=$1; LANES=$2; LIB=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$LIB" ] && export GGRS_AMD_EXP_LIB=$LIB
cd /tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY"
G2="SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS"
G3="SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_IFETCH_LEVEL"
G4="SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32"
for l in $LANES; do
  i=1
  for G in "$G1" "$G2" "$G3" "$G4"; do
    timeout -s KILL 90 rocprofv3 --pmc $G -d $OUT/l${l}_g$i -o pmc --output-format csv -- python3 $R/bench.py --no-cpu-baseline --lanes $l --steps 3 --warmup 1 > $OUT/l${l}_g$i.log 2>&1 || { echo "pass $l $i failed"; tail -5 $OUT/l${l}_g$i.log; exit 1; }
    i=$((i+1))
  done
  echo "lanes $l done"
done
