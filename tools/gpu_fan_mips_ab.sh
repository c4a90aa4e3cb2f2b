set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mips.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py > gpurun_out/fm_tests.log 2>&1 || { tail -30 gpurun_out/fm_tests.log; exit 1; }
tail -2 gpurun_out/fm_tests.log
rm -f gpurun_out/ab_summary.txt
REPS=2 BENCH_ARGS="--mode fan --mips --no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh tools/ubench/libgeo_fan2d.so tools/ubench/libgeo_fanmips2.so || exit 1
REPS=1 BENCH_ARGS="--mode fan --no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh tools/ubench/libgeo_fan2d.so tools/ubench/libgeo_fanmips2.so || exit 1
