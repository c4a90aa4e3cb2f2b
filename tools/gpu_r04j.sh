#!/bin/bash
# Session r04j: batched launches (geo_render_band_set_frames).  The GPU suite,
# then the host-bound probe per frame with and without batching for an
# N-rank share, a 2-rank gloo rehearsal of bench.py from one command
# (frame_check), and the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/r04j_gpu_suite.txt 2>&1 || { tail -30 $OUT/r04j_gpu_suite.txt; exit 1; }
tail -2 $OUT/r04j_gpu_suite.txt
for A in "8 1 8 2" "8 2 8 2" "4 1 8 2" "2 1 8 2" "8 1 8 1"; do
  for bt in 0 1; do
    timeout -k 10 200 python tools/host_bound_probe.py $A 400 $bt >> $OUT/r04j_host_probe.txt 2>&1 || { tail -5 $OUT/r04j_host_probe.txt; exit 1; }
  done
done
grep world $OUT/r04j_host_probe.txt
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --steps 40 --warmup 5 --no-cpu-baseline \
  > $OUT/r04j_gloo2.json 2> $OUT/r04j_gloo2.err || { tail -20 $OUT/r04j_gloo2.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/r04j_gloo2.json')); print('gloo2', d['world_size'], d['config']['frames_per_launch'], d['config']['rank0_lead'], d['frame_check'], round(d['ms_per_step'],4), d['kernel_ms']['events'][:60])"
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/r04j_cfg3.json 2> $OUT/r04j_cfg3.err || { tail -5 $OUT/r04j_cfg3.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/r04j_cfg3.json')); print('cfg3', round(d['ms_per_step'],5), round(d['kernel_ms']['avg'],5), round(d['roofline']['frac'],4), d['kernel_ms']['frames_timed'])"
