#!/bin/bash
# Sky-layout check + A/B: the GPU parity, fuzz and mips tests on the in-tree
# library, then bench.py on config 3 (direct) and fan mode over the libraries:
#   bash tools/gpu_sky_layout_ab.sh OLD.so NEW.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_mips.py > gpurun_out/layout_tests.log 2>&1 || { tail -30 gpurun_out/layout_tests.log; exit 1; }
tail -2 gpurun_out/layout_tests.log
rm -f gpurun_out/ab_summary.txt
REPS=${REPS:-3} BENCH_ARGS="--no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh "$@" || exit 1
REPS=2 BENCH_ARGS="--mode fan --no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh "$@" || exit 1
