#!/bin/bash
# The GPU suite, then bench lines: the default (metric) run and the
# mip-mapped sampler on configs 3 and 5 (context, not the metric).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --mips > gpurun_out/bench_${TAG}_mips.json 2> gpurun_out/bench_${TAG}_mips.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --mips --config cfg5_8k_adaptive --steps 100 > gpurun_out/bench_${TAG}_mips5.json 2> gpurun_out/bench_${TAG}_mips5.err || exit $?
echo ok
