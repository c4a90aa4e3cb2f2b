set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu_r01p.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu_r01p.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_points.py > gpurun_out/bench_points_r01p.json 2> gpurun_out/bench_points_r01p.err
rc=$?; cat gpurun_out/bench_points_r01p.json; tail -3 gpurun_out/bench_points_r01p.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_points.py --orbits --points 1000000 > gpurun_out/bench_points_orbits_r01p.json 2> gpurun_out/bench_points_orbits_r01p.err
rc=$?; cat gpurun_out/bench_points_orbits_r01p.json; tail -3 gpurun_out/bench_points_orbits_r01p.err; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_points_r01p" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_points.py" --cpu-connectors 200 > "$GRAFT_REPO_ROOT/gpurun_out/prof_points_r01p.log" 2>&1
echo "rocprof rc=$?"
