#!/bin/bash
# Focused GPU tests (given files), then the whole-tree check.  usage: bash tools/r03_focus.sh <tag> <test files...>
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_focus_$TAG.log 2>&1 || { echo "focused tests failed"; tail -50 gpurun_out/pytest_focus_$TAG.log; exit 10; }
tail -3 gpurun_out/pytest_focus_$TAG.log
