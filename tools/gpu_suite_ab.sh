#!/bin/bash
# The GPU suite on the in-tree library, then an A/B of prebuilt libraries
# (arguments) on configs 3 and 5, two interleaved repetitions each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_summary.txt
bash tools/gpu_ab_lib.sh "$@" || exit $?
BENCH_ARGS="--config cfg5_8k_adaptive --no-cpu-baseline --steps 200" bash tools/gpu_ab_lib.sh "$@"
