#!/bin/bash
# Fan kernel: GPU fan parity tests on the in-tree library, then
# tools/ubench/fan_time.py for each prebuilt library given (default: the
# literal and the latency-lean f64 loop).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fan" > gpurun_out/fanpar.log 2>&1; rc=$?
tail -2 gpurun_out/fanpar.log; [ $rc -eq 0 ] || exit $rc
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
cp "$LIB" gpurun_out/.libgeo_orig.so
[ $# -gt 0 ] || set -- tools/ubench/libgeo_fanlit.so tools/ubench/libgeo_fanfast.so
for rep in 1 2; do for v in "$@"; do
    cp "$v" "$LIB"
    FAN_LIB=$v timeout -k 10 120 python tools/ubench/fan_time.py || { cp gpurun_out/.libgeo_orig.so "$LIB"; exit 1; }
done; done
cp gpurun_out/.libgeo_orig.so "$LIB"
