#!/bin/bash
# Fan-draw variants (prebuilt libraries, the arguments): the fan-mode parity
# tests on each, then an interleaved A/B of bench.py --mode fan.
#   bash tools/gpu_fan_variants.sh TAG a.so b.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=$1; shift
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
cp $LIB $OUT/.libgeo_orig.so
for v in "$@"; do
  cp "$v" $LIB
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_tile_order.py -k fan -x -q \
      --timeout 120 --timeout-method thread > $OUT/fanpar_${TAG}_$(basename $v).log 2>&1 \
      || { tail -20 $OUT/fanpar_${TAG}_$(basename $v).log; cp $OUT/.libgeo_orig.so $LIB; exit 1; }
  echo "$v: $(tail -1 $OUT/fanpar_${TAG}_$(basename $v).log)"
done
rm -f $OUT/ab_summary.txt
REPS=${REPS:-3} BENCH_ARGS="--mode fan --no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh "$@" || exit 1
cp $OUT/ab_summary.txt $OUT/fanab_$TAG.txt
echo ok
