#!/bin/bash
# Session r04r: workgroup tile shape with the learned longest-first order
# (prebuilt variant libraries: waves abreast x tile rows), configs 2, 3 and
# the fan draw, interleaved, 2 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/ab_summary.txt
for C in "--config cfg2_1080p" "--config cfg3_4k" "--mode fan"; do
  echo "== $C" >> gpurun_out/ab_summary.txt
  REPS=2 BENCH_ARGS="$C --no-cpu-baseline --steps 300" bash tools/gpu_ab_lib.sh "$@" > /dev/null || exit 1
done
cp gpurun_out/ab_summary.txt gpurun_out/r04r_tile_ab.txt
cat gpurun_out/r04r_tile_ab.txt
