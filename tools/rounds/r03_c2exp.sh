#!/bin/bash
# Round 3: config-2 timing experiments: product at 512/1024/2048 frames per step, and timing builds
# under ggrs_amd/exp/ given as arguments (no parity).
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
run() {  # run <lib> <bench args>
  local lib=$1; shift
  GGRS_AMD_EXP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/b.json')); r=d.get('roofline') or {}; print(sys.argv[1] or 'product', sys.argv[2:], '%.4g'%d['value'], d['ms_per_step'], r.get('avg_launch_ms'))" "$lib" "$@" | tee -a gpurun_out/summary_$TAG.txt
}
run "" ; run "" --frames-per-step 1024; run "" --frames-per-step 2048
for L in "$@"; do run libggrs_amd_$L.so; done
