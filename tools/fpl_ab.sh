#!/bin/bash
# Frames per launch at N = 1 (bench.py --frames-per-launch K): K consecutive
# frames in one launch, interleaved A/B on one box.
#   bash tools/fpl_ab.sh TAG "cfg3_4k cfg2_1080p" "1 4 8" [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
: > "$OUT/fpl_ab.txt"
for rep in $(seq 1 ${4:-2}); do
  for c in $2; do
    for k in $3; do
      timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --steps 200 --frames-per-launch $k \
        > "$OUT/fpl.json" 2> "$OUT/fpl.err" || { tail -5 "$OUT/fpl.err"; exit 1; }
      python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1])
print('%-12s K=%s rep%s  ms/frame %.5f  kernel/frame %.5f  frac %.4f  value %.4g  frame_check %s' % (sys.argv[2], sys.argv[3], sys.argv[4], d['ms_per_step'], d['kernel_ms']['avg'], d['roofline']['frac'], d['value'], d['frame_check']['ok']))" \
        "$OUT/fpl.json" $c $k $rep | tee -a "$OUT/fpl_ab.txt"
    done
  done
done
