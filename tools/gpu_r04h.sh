#!/bin/bash
# Session r04h: (1) the GPU suite on the in-tree library (fan-buffer readers
# tracked by render slot on the writer's stream, no per-draw event work
# there); (2) A/B of the fan draw, previous vs current library; (3) what the
# in-region event pairs cost per frame: config 2 and the fan draw with event
# pairs on every 4th, 10th and only the first timed frame.
#   bash tools/gpu_r04h.sh tools/ubench/libgeo_prev.so tools/ubench/libgeo_cur.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04h_gpu_suite.txt 2>&1 || { tail -30 gpurun_out/r04h_gpu_suite.txt; exit 1; }
tail -2 gpurun_out/r04h_gpu_suite.txt
rm -f gpurun_out/ab_summary.txt
REPS=3 BENCH_ARGS="--mode fan --no-cpu-baseline --steps 400" bash tools/gpu_ab_lib.sh "$1" "$2" || exit $?
mv gpurun_out/ab_summary.txt gpurun_out/r04h_fan_chain_ab.txt
for rep in 1 2; do
  for cfg in "--config cfg2_1080p" "--mode fan"; do
    for ev in 4 10 100000; do
      timeout -k 10 300 python bench.py $cfg --no-cpu-baseline --steps 400 --event-every $ev > gpurun_out/ev.json 2> gpurun_out/ev.err \
        || { tail -5 gpurun_out/ev.err; exit 1; }
      python -c "
import json,sys; d=json.load(open('gpurun_out/ev.json'))
print('%-22s ev %-6s rep%s  ms/frame %.5f  compute-only %.5f  kernel avg %.5f (%d timed)' % (sys.argv[1], sys.argv[2], sys.argv[3],
      d['ms_per_step'], d['compute_only']['ms_per_step'], d['kernel_ms']['avg'], d['kernel_ms']['frames_timed']))
" "$cfg" "$ev" "$rep" | tee -a gpurun_out/r04h_event_cost.txt
    done
  done
done
