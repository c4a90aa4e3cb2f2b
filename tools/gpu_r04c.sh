#!/bin/bash
# Round-4 session c: the whole GPU suite on the tree with learned longest-first
# dispatch on by default, the dispatch-order probe, bench lines for configs
# 3, 2, 5 and rocprofv3 kernel stats for configs 2 and 5.
#   bash tools/gpu_r04c.sh TAG [--no-probe]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r04c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_$TAG.log" 2>&1 || { tail -30 "$OUT/pytest_$TAG.log"; exit 1; }
tail -2 "$OUT/pytest_$TAG.log"
if [ "${2:-}" != "--no-probe" ]; then
  timeout -k 10 600 python -u tools/order_probe.py cfg2_1080p cfg3_4k cfg5_8k_adaptive > "$OUT/order_$TAG.txt" 2>&1 \
      || { tail -5 "$OUT/order_$TAG.txt"; exit 1; }
  grep cfg "$OUT/order_$TAG.txt"
fi
for C in cfg3_4k cfg2_1080p cfg5_8k_adaptive; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline > "$OUT/bench_${TAG}_$C.json" 2> "$OUT/bench_${TAG}_$C.err" \
      || { tail -5 "$OUT/bench_${TAG}_$C.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_${TAG}_$C.json')); print('$C', round(d['ms_per_step'],5), round(d['kernel_ms']['avg'],5), round(d['roofline']['frac'],4), round(d['roofline']['frac_wall'],4))"
done
cd /tmp && export TMPDIR=/tmp
for C in cfg2_1080p cfg5_8k_adaptive cfg3_4k; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_$C" -o run \
      -- python3 "$ROOT/bench.py" --no-cpu-baseline --config $C > "$OUT/prof_${TAG}_$C.log" 2>&1 || exit 1
done
echo ok
