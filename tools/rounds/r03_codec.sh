#!/bin/bash
# codec: GPU tests, the bench in both layouts, trace + FETCH/WRITE PMC of the chunked default
# usage: bash tools/r03_codec.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_codec_$TAG.log 2>&1 || { echo "codec tests failed"; tail -40 gpurun_out/pytest_codec_$TAG.log; exit 10; }
tail -1 gpurun_out/pytest_codec_$TAG.log
for lay in chunked strided; do
  timeout -k 10 300 python -u bench.py --workload codec --no-cpu-baseline --codec-layout $lay > gpurun_out/codec_${TAG}_$lay.json 2> gpurun_out/codec_${TAG}_$lay.err || { tail -20 gpurun_out/codec_${TAG}_$lay.err; exit 11; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['kernel_ms'], d['roofline']['frac'], d['parity'])" gpurun_out/codec_${TAG}_$lay.json $lay
done
bash tools/profile.sh prof_codec_$TAG --workload codec || exit 12
echo codec done
