#!/bin/bash
# Round 4: the RayConnector throughput line (tools/bench_points.py, 2 M points,
# with and without orbits) on two libraries interleaved, then the gloo
# rehearsals of the multi-GPU bench on the in-tree library.
#   bash tools/gpu_r04p2.sh OLD.so NEW.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04p2
mkdir -p $OUT
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
LIBS=("$@")
cp "$LIB" $OUT/.orig.so
for rep in 1 2; do
  for v in "${LIBS[@]}"; do
    cp "$v" "$LIB"
    for o in "" "--orbits"; do
      timeout -k 10 180 python tools/bench_points.py $o --cpu-connectors 2000 > $OUT/p.json 2> $OUT/p.err \
        || { tail -5 $OUT/p.err; cp $OUT/.orig.so "$LIB"; exit 1; }
      python -c "
import json,sys; d=json.load(open('$OUT/p.json'))
print('%-16s rep%s %-9s %.4g %s  ms/step %.4f' % (sys.argv[1].split('/')[-1], sys.argv[2], sys.argv[3] or 'no-orbits', d['value'], d['unit'], d['ms_per_step']))
" "$v" "$rep" "$o" | tee -a $OUT/points_bench_ab.txt
    done
  done
done
cp $OUT/.orig.so "$LIB"
TAG=r04p2 bash tools/gpu_dist_rehearse.sh > $OUT/dist_rehearse.txt 2>&1 || { tail -5 $OUT/dist_rehearse.txt; exit 1; }
grep -c "frame-check" $OUT/dist_rehearse.txt
