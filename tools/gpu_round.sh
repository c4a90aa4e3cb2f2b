#!/bin/bash
# One GPU session: all GPU tests, smoke, a rendered frame, PMC passes for the
# config-3 and config-5 kernels (each its own rocprofv3 run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_$TAG.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/render_frame.py gpurun_out/frame_$TAG.png --width 960 --height 540 --frames 30 > gpurun_out/frame_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/frame_$TAG.log; [ $rc -eq 0 ] || exit $rc
SETS=("GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU" "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32" "SQ_THREAD_CYCLES_VALU SQ_WAVES" "SQ_INSTS_VALU_FLOPS_FP32" "FETCH_SIZE" "WRITE_SIZE")
CONFIG=cfg3_4k bash tools/gpu_pmc.sh pmc3_$TAG "${SETS[@]}" || exit $?
CONFIG=cfg5_8k_adaptive bash tools/gpu_pmc.sh pmc5_$TAG "${SETS[@]}" || exit $?
python tools/pmc_to_profile.py pmc3_$TAG gpurun_out/${TAG}_cfg3_4k_pmc.json "cfg3_4k (3840x2160, 2048 steps, direct)" > /dev/null
python tools/pmc_to_profile.py pmc5_$TAG gpurun_out/${TAG}_cfg5_8k_adaptive_pmc.json "cfg5_8k_adaptive (7680x4320, RK5(4) tol 1e-6, adaptive)" "geo_render_kernel<GEO_MODE_ADAPTIVE, kCurvedOut>"
