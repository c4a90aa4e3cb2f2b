#!/bin/bash
# Fan-mode draw check + A/B: the GPU parity and fuzz tests on the in-tree
# library, then bench.py --mode fan (config 3 4K) over the libraries given:
#   bash tools/gpu_fan_draw_ab.sh OLD.so NEW.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_mips.py > gpurun_out/fan_tests.log 2>&1 || { tail -20 gpurun_out/fan_tests.log; exit 1; }
tail -2 gpurun_out/fan_tests.log
rm -f gpurun_out/ab_summary.txt
REPS=${REPS:-3} BENCH_ARGS="--mode fan --no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh "$@" || exit 1
