#!/bin/bash
# The codec GPU tests on the product library, then old/new A/B pairs of the codec bench line
# (decode and encode kernel times by the bench's events).
set -e
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_codec.py -m gpu > gpurun_out/codec_tests.log 2>&1
tail -1 gpurun_out/codec_tests.log
for rep in 1 2 3; do
for lib in old new; do
  GGRS_AMD_EXP_LIB=libggrs_amd_$lib.so timeout -k 10 200 python -u bench.py --workload codec --steps 200 --no-cpu-baseline > gpurun_out/abc_${lib}_$rep.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/abc_${lib}_$rep.json').read().strip().splitlines()[-1]); print('$lib', d['value'], d['kernel_ms'], d['parity'])"
done
done
