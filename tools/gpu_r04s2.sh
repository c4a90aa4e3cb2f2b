#!/bin/bash
# Round 4: the disk update's size dispatch (fused for small clouds, orbit
# kernel + ray kernel for large ones) against the three-launch library: disk
# state byte for byte (small, changing dt, large), the points tests, the
# throughput line with and without orbits, the reference's fan-mode frame.
#   bash tools/gpu_r04s2.sh OLD.so NEW.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04s2
mkdir -p $OUT
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
OLD=$1; NEW=$2
cp "$LIB" $OUT/.orig.so
cp "$OLD" "$LIB"; timeout -k 10 180 python tools/points_dump.py $OUT/old.npz || { cp $OUT/.orig.so "$LIB"; exit 1; }
cp "$NEW" "$LIB"; timeout -k 10 180 python tools/points_dump.py $OUT/new.npz || { cp $OUT/.orig.so "$LIB"; exit 1; }
python -c "
import numpy as np; a = np.load('$OUT/old.npz'); b = np.load('$OUT/new.npz')
bad = [k for k in a.files if a[k].tobytes() != b[k].tobytes()]
print('disk state old vs new:', 'identical' if not bad else 'DIFFER in %s' % bad, '(%d arrays: %s)' % (len(a.files), ' '.join(a.files)))
raise SystemExit(1 if bad else 0)
" | tee $OUT/points_ab.txt || { cp $OUT/.orig.so "$LIB"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_parity.py -m gpu -x -q -k "point or disk or ray" \
  --timeout 120 --timeout-method thread > $OUT/pytest_points.log 2>&1
rc=$?; tail -1 $OUT/pytest_points.log; [ $rc -eq 0 ] || { cp $OUT/.orig.so "$LIB"; exit $rc; }
for rep in 1 2; do
  for v in "$OLD" "$NEW"; do
    cp "$v" "$LIB"
    for o in "" "--orbits"; do
      timeout -k 10 180 python tools/bench_points.py $o --cpu-connectors 2000 > $OUT/p.json 2> $OUT/p.err \
        || { tail -5 $OUT/p.err; cp $OUT/.orig.so "$LIB"; exit 1; }
      python -c "
import json,sys; d=json.load(open('$OUT/p.json'))
print('%-16s rep%s %-9s %.4g %s  ms/step %.4f' % (sys.argv[1].split('/')[-1], sys.argv[2], sys.argv[3] or 'no-orbits', d['value'], d['unit'], d['ms_per_step']))
" "$v" "$rep" "$o" | tee -a $OUT/ab.txt
    done
    timeout -k 10 120 python tools/bench_scene.py --mode fan --width 1920 --height 1080 --frames 400 > $OUT/s.json 2> $OUT/s.err \
      || { tail -5 $OUT/s.err; cp $OUT/.orig.so "$LIB"; exit 1; }
    python -c "
import json,sys; d=json.load(open('$OUT/s.json'))
print('%-16s rep%s scene fan 1080p ms/frame %.4f' % (sys.argv[1].split('/')[-1], sys.argv[2], d['ms_per_frame']))
" "$v" "$rep" | tee -a $OUT/ab.txt
  done
done
cp $OUT/.orig.so "$LIB"
