#!/bin/bash
# The P2P GPU tests on the product library, then old/new A/B pairs of the fixed-latency P2P lines
# (65,536 sessions; config 2's P2P shape) -- timing, parity legs on.
set -e
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_p2p.py tests/test_gpu_desync.py -m gpu > gpurun_out/p2p_tests.log 2>&1
tail -1 gpurun_out/p2p_tests.log
bash tools/ab_sched.sh "--workload p2p" old new
