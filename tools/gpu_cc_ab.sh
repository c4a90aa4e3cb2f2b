#!/bin/bash
# A/B of prebuilt libraries with the order probe (PROBE_ORDERS, default
# natural,auto) on the given specs: bash tools/gpu_cc_ab.sh TAG "specs" a.so b.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=$1; SPECS=$2; shift 2
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
cp $LIB $OUT/.libgeo_orig.so
for rep in 1 2; do
  for v in "$@"; do
    cp "$v" $LIB
    PROBE_ORDERS=${PROBE_ORDERS:-natural,auto} timeout -k 10 300 python -u tools/order_probe.py $SPECS > $OUT/cc.txt 2>&1 \
        || { tail -5 $OUT/cc.txt; cp $OUT/.libgeo_orig.so $LIB; exit 1; }
    grep cfg $OUT/cc.txt | sed "s|^|$(basename $v) rep$rep |" | tee -a $OUT/ccab_$TAG.txt
  done
done
cp $OUT/.libgeo_orig.so $LIB
