#!/bin/bash
# A/B kernel timing on the GPU box: rocprofv3 --kernel-trace --stats of one bench command per
# library, alternated twice (product library = "-", an experiment library = its basename under
# ggrs_amd/exp, selected through GGRS_AMD_EXP_LIB).
# usage: bash tools/ab_prof.sh <tag> "<bench args>" <lib> [<lib> ...]
set -u
TAG=$1; ARGS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for rep in 1 2; do
  for lib in "$@"; do
    name=${lib%.so}; [ "$lib" = "-" ] && name=product
    if [ "$lib" = "-" ]; then unset GGRS_AMD_EXP_LIB; else export GGRS_AMD_EXP_LIB=$lib; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${name}_$rep -o trace --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline $ARGS > $OUT/${name}_$rep.json 2> $OUT/${name}_$rep.err || { tail -20 $OUT/${name}_$rep.err; exit 1; }
    cat $OUT/${name}_$rep.json
  done
done
unset GGRS_AMD_EXP_LIB
echo ab done
