#!/bin/bash
# Long GPU fuzz sweeps on seeds beyond the committed ones (direct, adaptive,
# adversarial, fan, mips): each pytest run its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${N:-2000}
for t in "test_gpu_fuzz_bitexact" "test_gpu_fuzz_adversarial_bitexact" "test_gpu_fuzz_fan_mode_bitexact" "test_gpu_fuzz_mips_bitexact"; do
  GEO_FUZZ_N=$N GEO_FUZZ_BASE=${BASE:-200000} timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -s \
      -k "$t" --timeout 850 --timeout-method thread > gpurun_out/fuzz_$t.log 2>&1
  rc=$?; grep -h "^fuzz" gpurun_out/fuzz_$t.log; tail -1 gpurun_out/fuzz_$t.log
  [ $rc -eq 0 ] || exit $rc
done
