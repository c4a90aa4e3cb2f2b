#!/bin/bash
# Session r04l: rank 0's share as a ratio of bands (BandLayout peer_bands,
# geo_assemble_shares, bench.py --rank0-lead a:b): the pipeline and assembly
# GPU tests, then gloo rehearsals of bench.py with 3:2 and auto (8 layouts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_pipeline.py tests/test_gpu_batch.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $OUT/r04l_tests.txt 2>&1 || { tail -30 $OUT/r04l_tests.txt; exit 1; }
tail -1 $OUT/r04l_tests.txt
for spec in "2 3:2 20" "3 5:2 12" "3 auto 30" "2 1:2 9"; do
  set -- $spec
  timeout -k 10 300 python bench.py --gpus $1 --steps $3 --warmup 2 --spinup-frames 2 --no-cpu-baseline \
      --dist-backend gloo --rank0-lead $2 --lead-trial-frames 8 > $OUT/r04l_gloo_$1_${2/:/_}.json 2> $OUT/r04l_gloo_$1_${2/:/_}.err \
      || { tail -10 $OUT/r04l_gloo_$1_${2/:/_}.err; exit 1; }
  python -c "
import json,sys; d=json.load(open(sys.argv[1])); c=d['config']
print('gloo world', d['world_size'], 'lead', c['rank0_lead'], 'trials', c['lead_trials_ms_per_frame'] and sorted(c['lead_trials_ms_per_frame']), 'batch', c['frames_per_launch'], d['frame_check']['ok'], d['frame_check']['frames'])" $OUT/r04l_gloo_$1_${2/:/_}.json
done
