#!/bin/bash
# Session r04n: issue priority for long-running waves (GEO_PRIO_STEPS A/B,
# prebuilt libraries): configs 2, 3 and 5, interleaved, 2 reps each.
#   bash tools/gpu_r04n.sh LIB...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/ab_summary.txt
for C in cfg2_1080p cfg3_4k cfg5_8k_adaptive; do
  echo "== $C" >> gpurun_out/ab_summary.txt
  REPS=2 BENCH_ARGS="--config $C --no-cpu-baseline --steps 300" bash tools/gpu_ab_lib.sh "$@" > /dev/null || exit 1
done
cp gpurun_out/ab_summary.txt gpurun_out/r04n_prio_ab.txt
cat gpurun_out/r04n_prio_ab.txt
