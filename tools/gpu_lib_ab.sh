#!/bin/bash
# GPU parity tests on the in-tree library, then an A/B of prebuilt libraries
# (the arguments; default tools/ubench/libgeo_prev.so tools/ubench/libgeo_cur.so)
# on configs 3 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?
tail -2 gpurun_out/par.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_summary.txt
[ $# -gt 0 ] || set -- tools/ubench/libgeo_prev.so tools/ubench/libgeo_cur.so
bash tools/gpu_ab_lib.sh "$@" || exit $?
BENCH_ARGS="--config cfg5_8k_adaptive --no-cpu-baseline --steps 200" bash tools/gpu_ab_lib.sh "$@"
