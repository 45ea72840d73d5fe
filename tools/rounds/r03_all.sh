#!/bin/bash
# Round 3 whole-tree pass: GPU tests, smoke, every workload's bench line, config-3 and P2P profiles.
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 11; }
tail -1 gpurun_out/smoke_$TAG.log
i=0
for a in "" "--config 3" "--config 4" "--config 5" "--workload p2p" "--workload p2p --sparse" "--workload codec" "--workload requests" "--workload requests --req-groups 4"; do
  timeout -k 10 300 python -u bench.py $a > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err || { echo "bench '$a' failed"; tail -20 gpurun_out/bench_${TAG}_$i.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2] or 'config2', '%.4g'%d['value'], d['ms_per_step'], r.get('frac'), (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/bench_${TAG}_$i.json "$a"
  i=$((i+1))
done
bash tools/profile.sh ${TAG}_c3 --config 3 --steps 10 || exit 13
bash tools/profile.sh ${TAG}_p2p --workload p2p --steps 10 || exit 14
echo all done
