#!/bin/bash
# Round-4 session b: the tile-order tests, the dispatch-order probe (configs
# 2, 3, 5 and the fan draw), and an A/B of the library before/after the
# tile-order hook (tools/ubench/libgeo_prev.so vs libgeo_cur.so) on configs 3 and 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r04b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_tile_order.py -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_$TAG.log" 2>&1 || { tail -30 "$OUT/pytest_$TAG.log"; exit 1; }
tail -2 "$OUT/pytest_$TAG.log"
timeout -k 10 600 python -u tools/order_probe.py cfg2_1080p cfg3_4k cfg5_8k_adaptive cfg3_4k:fan > "$OUT/order_$TAG.txt" 2>&1 \
    || { tail -5 "$OUT/order_$TAG.txt"; exit 1; }
cat "$OUT/order_$TAG.txt"
rm -f "$OUT/ab_summary.txt"
BENCH_ARGS="--no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh tools/ubench/libgeo_prev.so tools/ubench/libgeo_cur.so || exit 1
BENCH_ARGS="--config cfg2_1080p --no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh tools/ubench/libgeo_prev.so tools/ubench/libgeo_cur.so || exit 1
echo ok
