#!/bin/bash
# PMC passes (tools/gpu_pmc.sh) for the in-tree library and for a prebuilt
# variant (tools/build_variant.py), one after the other on one box; the
# in-tree library is restored after.
#   VARIANT=tools/ab/x.so CONFIG=cfg3_4k [EXTRA_ARGS="--mode fan"] bash tools/pmc_variant_probe.sh TAG "SET1" ["SET2" ...]
# Output: gpurun_out/TAG_orig_<i>/, gpurun_out/TAG_variant_<i>/ (run_counter_collection.csv).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
cp "$LIB" /tmp/pmc_variant_orig.so
bash tools/gpu_pmc.sh "${TAG}_orig" "$@" || exit $?
cp "$VARIANT" "$LIB"
bash tools/gpu_pmc.sh "${TAG}_variant" "$@"
rc=$?
cp /tmp/pmc_variant_orig.so "$LIB"
exit $rc
