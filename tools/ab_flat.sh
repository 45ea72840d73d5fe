#!/bin/bash
# The scheduled P2P tests, then old/new A/B pairs of the flat kernel's lines (65,536 sessions:
# jitter and stall).  Timing only for the A/B; the tests run on the product library.
set -e
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_p2p_sched.py tests/test_gpu_sched_desync.py -m gpu > gpurun_out/sched_tests_flat.log 2>&1
tail -1 gpurun_out/sched_tests_flat.log
bash tools/ab_sched.sh "--workload p2p --arrivals jitter" old new
bash tools/ab_sched.sh "--workload p2p --arrivals stall" old new
