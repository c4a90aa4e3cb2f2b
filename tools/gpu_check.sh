#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace profile.
# Each GPU step has its own time limit; a crash/timeout (exit >= 124 or a
# signal) ends the script, a plain test failure (pytest exit 1) does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r01}

fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -ge 128 ]; }

GEO_F64_BAR_OUT="$OUT/f64bar_$TAG" timeout -k 10 420 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu_$TAG.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke_$TAG.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

timeout -k 10 300 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_$TAG.json"; tail -3 "$OUT/bench_$TAG.err"
if [ $rc -ne 0 ]; then exit $rc; fi

# further configs (e.g. EXTRA_CONFIGS="cfg5_8k_adaptive"): bench line each
for C in ${EXTRA_CONFIGS:-}; do
    timeout -k 10 300 python bench.py --config "$C" > "$OUT/bench_${TAG}_$C.json" 2> "$OUT/bench_${TAG}_$C.err"
    rc=$?; echo "bench $C rc=$rc"; cat "$OUT/bench_${TAG}_$C.json"; tail -3 "$OUT/bench_${TAG}_$C.err"
    if [ $rc -ne 0 ]; then exit $rc; fi
done

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof_$TAG.log"
if [ $rc -ne 0 ]; then exit $rc; fi
for C in ${EXTRA_CONFIGS:-}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_$C" -o run \
        -- python3 "$ROOT/bench.py" --no-cpu-baseline --config "$C" > "$OUT/prof_${TAG}_$C.log" 2>&1
    rc=$?; echo "rocprof $C rc=$rc"; tail -3 "$OUT/prof_${TAG}_$C.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
