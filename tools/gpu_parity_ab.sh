#!/bin/bash
# GPU parity tests on the in-tree library, then an A/B of compile-time variants.
#   bash tools/gpu_parity_ab.sh "-DX=0" "-DX=1"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/parity_ab_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/parity_ab_pytest.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_summary.txt
[ $# -gt 0 ] && bash tools/gpu_ab.sh "$@"
