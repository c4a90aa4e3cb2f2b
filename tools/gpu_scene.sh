#!/bin/bash
# The whole reference frame on one GPU: GPU tests of the point path and the
# C++ host, then tools/bench_scene.py with the disk update overlapped (side
# stream) and not, at 4K and 1080p, and the C++ frame loop both ways.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r01}
timeout -k 10 300 python -u -m pytest tests/test_gpu_points.py tests/test_cpp_host.py tests/test_gpu_parity.py -m gpu -q -rf -x \
    --timeout 120 --timeout-method thread > $OUT/pytest_scene_$TAG.log 2>&1
rc=$?; tail -4 $OUT/pytest_scene_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for S in 1 3; do for OV in 0 1; do for WH in "3840 2160" "1920 1080"; do
    set -- $WH
    timeout -k 10 120 python tools/bench_scene.py --width $1 --height $2 --spheres $S --overlap $OV \
        > $OUT/scene_${TAG}_s${S}_o${OV}_$2.json 2> $OUT/scene_${TAG}_s${S}_o${OV}_$2.err
    rc=$?; echo "scene s=$S overlap=$OV ${1}x$2 rc=$rc"; cat $OUT/scene_${TAG}_s${S}_o${OV}_$2.json; [ $rc -eq 0 ] || exit $rc
done; done; done
# the reference's display path: per-frame f64 fans + fan-lerp draws
for S in 1 3; do for WH in "3840 2160" "1920 1080"; do
    set -- $WH
    timeout -k 10 120 python tools/bench_scene.py --mode fan --width $1 --height $2 --spheres $S --overlap 1 \
        > $OUT/scene_${TAG}_fan_s${S}_$2.json 2> $OUT/scene_${TAG}_fan_s${S}_$2.err
    rc=$?; echo "scene fan s=$S ${1}x$2 rc=$rc"; cat $OUT/scene_${TAG}_fan_s${S}_$2.json; [ $rc -eq 0 ] || exit $rc
done; done
g++ -std=c++17 -O2 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include examples/frame_loop.cpp \
    -L schwarzschild_raytracer_wgpu_amd -lgeo -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,$(pwd)/schwarzschild_raytracer_wgpu_amd \
    -Wl,-rpath,/opt/rocm/lib -o $OUT/frame_loop || exit 1
for OV in 1 0; do
    timeout -k 10 120 $OUT/frame_loop 3840 2160 1000 $OUT/fl4k_$OV.ppm $OV >> $OUT/frame_loop_$TAG.txt || exit $?
    timeout -k 10 120 $OUT/frame_loop 1920 1080 2000 $OUT/fl1080_$OV.ppm $OV >> $OUT/frame_loop_$TAG.txt || exit $?
done
for WH in "3840 2160" "1920 1080"; do
    set -- $WH
    timeout -k 10 120 $OUT/frame_loop $1 $2 2000 $OUT/flfan1_$2.ppm 1 fan >> $OUT/frame_loop_$TAG.txt || exit $?
    timeout -k 10 120 $OUT/frame_loop $1 $2 2000 $OUT/flfan0_$2.ppm 0 fan >> $OUT/frame_loop_$TAG.txt || exit $?
    cmp $OUT/flfan1_$2.ppm $OUT/flfan0_$2.ppm || { echo "fan-mode frames differ"; exit 1; }
done
cat $OUT/frame_loop_$TAG.txt
cmp $OUT/fl4k_0.ppm $OUT/fl4k_1.ppm && cmp $OUT/fl1080_0.ppm $OUT/fl1080_1.ppm && echo "frames equal"
rm -f $OUT/fl*.ppm
