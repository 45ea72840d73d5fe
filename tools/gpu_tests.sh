#!/bin/bash
# Run a subset of GPU tests on the box: bash tools/gpu_tests.sh <tag> <pytest args...>
TAG=$1; shift
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out && timeout -k 10 500 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_$TAG.log; exit $rc
