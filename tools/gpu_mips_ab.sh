#!/bin/bash
# GEO_FLAG_MIPS check + A/B: the mips GPU tests on the in-tree library, then
# bench.py --mips (config 3, config 5) over the libraries given:
#   bash tools/gpu_mips_ab.sh OLD.so NEW.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mips.py tests/test_gpu_fuzz.py -k "mips" > gpurun_out/mips_tests.log 2>&1 || { tail -20 gpurun_out/mips_tests.log; exit 1; }
tail -2 gpurun_out/mips_tests.log
rm -f gpurun_out/ab_summary.txt
REPS=2 BENCH_ARGS="--mips --no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh "$@" || exit 1
REPS=1 BENCH_ARGS="--config cfg5_8k_adaptive --mips --no-cpu-baseline --steps 200" bash tools/gpu_ab_lib.sh "$@" || exit 1
