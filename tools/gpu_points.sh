#!/bin/bash
# The accretion-disk point path on one GPU: GPU tests, tools/bench_points.py
# (connectors; f64 orbits), rocprofv3 kernel stats, and the FETCH_SIZE /
# WRITE_SIZE passes (each its own run) summarised into <TAG>_points_pmc.json.
#   bash tools/gpu_points.sh r02p
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
TAG=${1:-r02p}
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_${TAG}.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_points.py > gpurun_out/bench_points_${TAG}.json 2> gpurun_out/bench_points_${TAG}.err
rc=$?; cat gpurun_out/bench_points_${TAG}.json; tail -3 gpurun_out/bench_points_${TAG}.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_points.py --orbits --points 1000000 > gpurun_out/bench_points_orbits_${TAG}.json 2> gpurun_out/bench_points_orbits_${TAG}.err
rc=$?; cat gpurun_out/bench_points_orbits_${TAG}.json; tail -3 gpurun_out/bench_points_orbits_${TAG}.err; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_points_${TAG}" -o run -- python3 "$ROOT/tools/bench_points.py" --cpu-connectors 200 > "$ROOT/gpurun_out/prof_points_${TAG}.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$ROOT/gpurun_out/pmcp_${TAG}_$C" -o run -- python3 "$ROOT/tools/bench_points.py" --cpu-connectors 200 --steps 20 > "$ROOT/gpurun_out/pmcp_${TAG}_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd "$ROOT"
python - "$TAG" <<'PY'
import glob, json, sys
sys.path.insert(0, "tools")
from pmc_summary import load
tag = sys.argv[1]
c = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/pmcp_{tag}_{ctr}/**/run_counter_collection.csv", recursive=True)[0]
    cc, _ = load(f, kernel="geo_rays_kernel<false>")
    c.update(cc)
n = 2 * (1 << 21)
rd, wr = 2.0 * c["FETCH_SIZE"] * 1024.0, c["WRITE_SIZE"] * 1024.0
out = {"kernel": "geo_rays_kernel<false> (RayConnector update_ray(observer, 1))",
       "workload": f"{n} connectors ({n // 2} points x 2 sides), 48 nodes",
       "source": f"rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over tools/bench_points.py, gpurun_out/pmcp_{tag}_*",
       "counters_per_dispatch": c,
       "derived": {"hbm_read_bytes": rd, "hbm_write_bytes": wr, "traffic_bytes": rd + wr,
                   "algorithmic_bytes": 408.0 * n,
                   "note": "reads are 16-B/lane streaming loads: FETCH_SIZE reports half their bytes on gfx950 "
                           "(MI355X_MICROARCH.md, HBM section), so it is doubled; WRITE_SIZE is exact for 16-B/lane stores"}}
json.dump(out, open(f"gpurun_out/{tag}_points_pmc.json", "w"), indent=1)
print(json.dumps(out["derived"], indent=1))
PY
