#!/bin/bash
# Round 4: codec decode (prefetched length / reference, whole-row writes, reused output); codec GPU tests and bench
# line (twice); config 4 and config 3 (general form) after the rounds_kernel experiment's removal.
set -u
TAG=${1:-r04l}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_codec.py \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err \
    || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; r=d.get('roofline') or {}; print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'], r.get('avg_launch_ms'), c.get('general_form_frames_per_s', ''))" gpurun_out/bench_${TAG}_$name.json $name
}
run codec_1 --workload codec
run codec_2 --workload codec
run c4_1 --config 4
run c3_1 --config 3
bash tools/profile.sh ${TAG}_codec --workload codec || exit 12
echo $TAG done
