#!/bin/bash
# Round 3: the magic-number sincos reduction (product) vs timing builds (ggrs_amd/exp/): the
# max-ilp machine scheduler (ilp), next-step sincos pinned before the clamp branch (pin), both.
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sincosf.py tests/test_gpu_synctest.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -1 gpurun_out/pytest_$TAG.log
run() {  # run <workload args> <lib>
  GGRS_AMD_EXP_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline $1 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/b.json')); r=d.get('roofline') or {}; print(sys.argv[1] or 'config2', sys.argv[2] or 'product', '%.4g'%d['value'], d['ms_per_step'], r.get('avg_launch_ms', r.get('avg_kernel_ms_per_round')), d.get('parity'))" "$1" "$2" | tee -a gpurun_out/summary_$TAG.txt
}
for LIB in "" libggrs_amd_ilp.so libggrs_amd_pin.so libggrs_amd_pinilp.so "" libggrs_amd_ilp.so libggrs_amd_pin.so libggrs_amd_pinilp.so; do run "" "$LIB"; done
for W in "--config 3" "--config 4" "--workload p2p" "--workload requests"; do
  for LIB in "" libggrs_amd_ilp.so; do run "$W" "$LIB"; done
done
