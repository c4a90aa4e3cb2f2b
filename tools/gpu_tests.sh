#!/bin/bash
# The GPU test suite on the in-tree library (one process, per-test timeout).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?
tail -3 gpurun_out/par.log; exit $rc
