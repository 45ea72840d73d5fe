#!/bin/bash
# gpurun wrapper for this session: retries ONLY when gpurun reports that nothing ran (infrastructure
# "transient" status or exit code 3 = no box free); a command that ran is never retried.
# usage: tools/gpu.sh <timeout_s> '<command>'
T=$1; shift
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$rc" = "3" ] || [ "$st" = "transient" ]; then
    echo "[gpu.sh] nothing ran (rc=$rc status=$st); retry $attempt in 40s" >&2
    sleep 40
    continue
  fi
  exit $rc
done
exit 3
