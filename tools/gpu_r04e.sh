#!/bin/bash
# Round-4 session e: dispatch-attached timing (tests, bench vs rocprofv3 on
# config 3), and the cost-class resolution A/B on config 2 and on 8- and
# 4-rank shares of config 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r04e}
timeout -k 10 300 python -u -m pytest tests/test_gpu_tile_order.py tests/test_bench.py -x -q --timeout 200 \
    --timeout-method thread > "$OUT/pytest_$TAG.log" 2>&1 || { tail -30 "$OUT/pytest_$TAG.log"; exit 1; }
tail -1 "$OUT/pytest_$TAG.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_${TAG}_cfg3.json" 2> "$OUT/bench_${TAG}_cfg3.err" || exit 1
python -c "import json; d=json.load(open('$OUT/bench_${TAG}_cfg3.json')); print('cfg3', round(d['ms_per_step'],5), d['kernel_ms'], round(d['roofline']['frac'],4))"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_cfg3" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/prof_${TAG}_cfg3.log" 2>&1) || exit 1
python tools/trace_window.py "$OUT/prof_${TAG}_cfg3/run_kernel_trace.csv" | tail -3
grep -h '^{' "$OUT/prof_${TAG}_cfg3.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('under rocprof: bench kernel avg', d['kernel_ms']['avg'])"
PROBE_ORDERS=natural,auto,lpt bash tools/gpu_cc_ab.sh $TAG "cfg2_1080p cfg3_4k@8 cfg3_4k@4" \
    tools/ubench/libgeo_cc1.so tools/ubench/libgeo_cc2.so tools/ubench/libgeo_cc3.so || exit 1
echo ok
