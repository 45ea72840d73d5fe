#!/bin/bash
# Scheduler-strategy A/B of the scheduled kernels: 4,096-session jitter (chains) and 65,536-session
# jitter (flat), libraries from ggrs_amd/exp (timing only).
cd ${GRAFT_REPO_ROOT:-.}
bash tools/ab_sched.sh "--workload p2p --arrivals jitter --sessions 4096 --max-prediction 9" "$@" || exit 1
bash tools/ab_sched.sh "--workload p2p --arrivals jitter" "$@"
