#!/bin/bash
# PMC counter passes (each its own rocprofv3 run, kernel-trace only, no sys/runtime trace).
#   CONFIG=cfg5_8k_adaptive [EXTRA_ARGS="--mode fan"] bash tools/gpu_pmc.sh TAG "SET1" "SET2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-pmc}
shift || true
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d "$OUT/${TAG}_$i" -o run \
     -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --spinup-frames 10 --no-cpu-baseline --config "${CONFIG:-cfg3_4k}" ${EXTRA_ARGS:-} > "$OUT/${TAG}_$i.log" 2>&1
  rc=$?; echo "pass $i ($SET) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/${TAG}_$i.log"; exit $rc; fi
done
