#!/bin/bash
# The P2P request encoder's thread scaling on the GPU box, with the cgroup's CPU quota and its
# throttling counters around each run: bash tools/req_plateau.sh <tag> "<env + bench args>" ...
TAG=$1; shift
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
OUT=gpurun_out/plateau_$TAG.txt
CG=/sys/fs/cgroup
{
  echo "nproc $(nproc) affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
  echo "cpu.max: $(cat $CG/cpu.max 2>/dev/null || echo n/a)"
  lscpu 2>/dev/null | grep -E "Model name|Socket|Core|Thread|L3|NUMA node\(s\)" || true
} > $OUT
i=0
for a in "$@"; do
  s0=$(cat $CG/cpu.stat 2>/dev/null | tr '\n' ' ')
  timeout -k 10 300 env $a > gpurun_out/plateau_${TAG}_$i.json 2> gpurun_out/plateau_${TAG}_$i.err || { echo "run '$a' failed" >> $OUT; tail -5 gpurun_out/plateau_${TAG}_$i.err >> $OUT; exit 1; }
  s1=$(cat $CG/cpu.stat 2>/dev/null | tr '\n' ' ')
  echo "RUN $i: $a" >> $OUT
  echo "  cpu.stat before: $s0" >> $OUT
  echo "  cpu.stat after:  $s1" >> $OUT
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('  value', d['value'], 'us_per_call', d['config']['us_per_call'], 'phases', d['config'].get('us_per_call_encode_handback_submit_wait_session'), 'profile', json.dumps(d.get('host_profile')))" gpurun_out/plateau_${TAG}_$i.json >> $OUT
  i=$((i+1))
done
cat $OUT
