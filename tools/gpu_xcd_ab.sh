#!/bin/bash
# GPU parity on the in-tree library, then the XCD-remap A/B: prebuilt
# libraries (GEO_XCD_CHUNK 1 / 4 / 8, tools/build_variant.py) timed
# interleaved on configs 3, 5 and 2, and one PMC pass each for the render
# kernel's L2->fabric read requests by size (read bytes = 64 n64 + 128 n128;
# FETCH_SIZE counts a 128-B request as 64 B on gfx950, tools/ubench/fetch_calib.hip).
#   bash tools/gpu_xcd_ab.sh tools/ubench/libgeo_x1.so tools/ubench/libgeo_x4.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?
tail -2 gpurun_out/par.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_summary.txt
bash tools/gpu_ab_lib.sh "$@" || exit $?
BENCH_ARGS="--config cfg5_8k_adaptive --no-cpu-baseline --steps 200" bash tools/gpu_ab_lib.sh "$@" || exit $?
BENCH_ARGS="--config cfg2_1080p --no-cpu-baseline --steps 1000" bash tools/gpu_ab_lib.sh "$@" || exit $?
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
cp "$LIB" gpurun_out/.libgeo_orig.so
i=0
for v in "$@"; do
  i=$((i+1)); cp "$v" "$LIB"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace \
     --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum WRITE_SIZE --output-format csv -d "$ROOT/gpurun_out/xab/v$i" -o run \
     -- python3 "$ROOT/bench.py" --steps 20 --warmup 2 --spinup-frames 10 --no-cpu-baseline > "$ROOT/gpurun_out/xab_v$i.log" 2>&1) \
     || { tail -5 gpurun_out/xab_v$i.log; cp gpurun_out/.libgeo_orig.so "$LIB"; exit 1; }
  python - "gpurun_out/xab/v$i" "$v" <<'PY'
import glob, sys
sys.path.insert(0, "tools")
from pmc_summary import load
c, d = load(glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0], kernel="geo_render")
rd = 64 * c["TCC_EA0_RDREQ_64B_sum"] + 128 * c["TCC_EA0_RDREQ_128B_sum"]
print(f"{sys.argv[2]:40s} read {rd / 1e6:.1f} MB  write {c['WRITE_SIZE'] * 1024 / 1e6:.1f} MB  dispatch {sum(d.values()) / len(d) / 1e3:.1f} us")
PY
done
cp gpurun_out/.libgeo_orig.so "$LIB"
