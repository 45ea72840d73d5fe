#!/bin/bash
# Config-5 sweep on the GPU box: particle parity tests, then the config-5 bench per entities-per-thread form.
# usage: bash tools/c5_sweep.sh [EPT values...]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_particles.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_pw.log 2>&1 || { tail -30 gpurun_out/t_pw.log; exit 10; }
tail -2 gpurun_out/t_pw.log
for e in ${@:-1 2 4}; do
  GGRS_PW_EPT=$e timeout -k 10 200 python -u bench.py --config 5 --no-cpu-baseline > gpurun_out/b_c5_e$e.json 2> gpurun_out/b_c5_e$e.err || { tail gpurun_out/b_c5_e$e.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/b_c5_e$e.json'));print($e, d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
