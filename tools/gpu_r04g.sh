#!/bin/bash
# Session r04g: the fan-mode draw with 4 pixels per lane (GEO_FAN_LR=4).
# The fan-mode GPU tests with the candidate library in place of the in-tree
# one, then an interleaved A/B of the fan draw (4K) against 2 pixels per lane.
#   bash tools/gpu_r04g.sh tools/ubench/libgeo_lr2.so tools/ubench/libgeo_lr4.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
cp "$LIB" gpurun_out/.libgeo_intree.so
cp "$2" "$LIB"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_cpu_path.py tests/test_gpu_dist_pipeline.py \
  > gpurun_out/r04g_tests_cand.log 2>&1; rc=$?
cp gpurun_out/.libgeo_intree.so "$LIB"
tail -3 gpurun_out/r04g_tests_cand.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_summary.txt
REPS=${REPS:-3} BENCH_ARGS="--mode fan --no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh "$1" "$2" || exit $?
cp gpurun_out/ab_summary.txt gpurun_out/r04g_fan_lr_ab.txt
