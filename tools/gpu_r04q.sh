#!/bin/bash
# Session r04q: gloo rehearsals of bench.py across modes and configs at
# N = 2, 3 (one GPU, host-staged gathers): config 2, config 5 (adaptive, 8K),
# the fan-mode draw, batched launches on and off, fixed and auto shares;
# every line's frame_check must hold.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/r04q_rehearsals.txt
for spec in "2 cfg2_1080p direct on auto 20" "3 cfg2_1080p direct off 3:2 12" "2 cfg5_8k_adaptive adaptive on 2 8" \
            "2 cfg3_4k fan on auto 16" "3 cfg3_4k fan off 1:2 9" "3 cfg3_4k direct on 5:2 24"; do
  set -- $spec
  timeout -k 10 300 python bench.py --gpus $1 --config $2 --mode $3 --batch-launch $4 --rank0-lead $5 --steps $6 \
      --warmup 2 --spinup-frames 2 --no-cpu-baseline --dist-backend gloo --lead-trial-frames 8 \
      > $OUT/r04q.json 2> $OUT/r04q.err || { tail -10 $OUT/r04q.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('$OUT/r04q.json')); c=d['config']; f=d['frame_check']
print('N=%s %s %s batch=%s lead=%s steps=%s -> frames_per_launch %s rank0_lead %s frame_check %s (%d frames)' % (tuple(sys.argv[1:]) + (c['frames_per_launch'], c['rank0_lead'], f['ok'], f['frames'])))
assert f['ok']" $@ | tee -a $OUT/r04q_rehearsals.txt || exit 1
done
