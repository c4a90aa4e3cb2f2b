#!/bin/bash
# The GPU suite with a prebuilt candidate library in place of the in-tree one,
# then an interleaved A/B of the two on configs 3 and 5.
#   REPS=3 bash tools/gpu_lib_parity_ab.sh base.so cand.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
cp "$LIB" gpurun_out/.libgeo_intree.so
cp "$2" "$LIB"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_cand.log 2>&1; rc=$?
cp gpurun_out/.libgeo_intree.so "$LIB"
tail -3 gpurun_out/pytest_gpu_cand.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_summary.txt
bash tools/gpu_ab_lib.sh "$1" "$2" || exit $?
BENCH_ARGS="--config cfg5_8k_adaptive --no-cpu-baseline --steps 200" bash tools/gpu_ab_lib.sh "$1" "$2"
