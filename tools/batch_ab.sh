#!/bin/bash
# Batched-launch A/B of prebuilt libraries (LIBS="a.so b.so"): an 8-rank share
# of config 3 alone in launches of 8 frames (--share 1/8), and the full
# config-3 and config-5 frames at 8 frames per launch; interleaved.
#   LIBS="a.so b.so" bash tools/batch_ab.sh TAG [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
cp "$LIB" "$OUT/.orig.so"
: > "$OUT/batch_ab.txt"
for rep in $(seq 1 ${2:-2}); do
  for spec in "--share 1/8 --frames-per-gather 8 --batch-launch on" "--frames-per-launch 8" \
              "--config cfg5_8k_adaptive --frames-per-launch 8"; do
    for v in $LIBS; do
      cp "$v" "$LIB"
      timeout -k 10 300 python3 bench.py $spec --no-cpu-baseline --steps 200 > "$OUT/b.json" 2> "$OUT/b.err" \
        || { tail -5 "$OUT/b.err"; cp "$OUT/.orig.so" "$LIB"; exit 1; }
      python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1])
print('%-52s %-22s rep%s  ms/frame %.5f  kernel/frame %.5f' % (sys.argv[2], sys.argv[3].split('/')[-1], sys.argv[4], d['ms_per_step'], d['kernel_ms']['avg']))" \
        "$OUT/b.json" "$spec" "$v" "$rep" | tee -a "$OUT/batch_ab.txt"
    done
  done
done
cp "$OUT/.orig.so" "$LIB"
