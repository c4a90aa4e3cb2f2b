#!/bin/bash
# Round 4 (v): per-kernel times of the reference's fan-mode frame (1080p,
# tools/bench_scene.py) under rocprofv3 for each library given, the disk state
# of each against the first byte for byte (tools/points_dump.py), then frame
# times interleaved.
#   bash tools/gpu_r04v.sh BASE.so A.so [B.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04v
mkdir -p $OUT
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
cp "$LIB" $OUT/.orig.so
export TMPDIR=/tmp
i=0
for v in "$@"; do
  cp "$v" "$LIB"
  timeout -k 10 120 python tools/points_dump.py $OUT/points_$i.npz || { cp $OUT/.orig.so "$LIB"; exit 1; }
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$i -o scene -- python3 tools/bench_scene.py \
    --mode fan --width 1920 --height 1080 --frames 300 > $OUT/traced_$i.json 2> $OUT/prof_$i.err \
    || { tail -5 $OUT/prof_$i.err; cp $OUT/.orig.so "$LIB"; exit 1; }
  python - "$v" $OUT/prof_$i <<'PY' | tee -a $OUT/kernels.txt
import glob, sqlite3, sys
db = glob.glob(sys.argv[2] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
print(sys.argv[1])
for name, calls, total, avg, pct in c.execute("select * from top_kernels"):
    print("  %-70s calls %5d  avg %8.2f us" % (name[:70], calls, avg))
PY
  python -c "
import numpy as np; a = np.load('$OUT/points_0.npz'); b = np.load('$OUT/points_$i.npz')
bad = [k for k in a.files if a[k].tobytes() != b[k].tobytes()]
print('  disk state vs the first library:', 'identical' if not bad else 'DIFFER in %s' % bad)
if bad:
    for k in bad:
        x, y = a[k].astype(np.float64), b[k].astype(np.float64)
        print('    %s: %d of %d values differ, max |diff| %.3g' % (k, int((x != y).sum()), x.size, float(np.abs(x - y).max())))
" | tee -a $OUT/kernels.txt
  i=$((i + 1))
done
# the last library against the oracle (orbits to a tolerance, connectors and draws bit for bit)
timeout -k 10 300 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_parity.py -m gpu -x -q -k "point or disk or ray" \
  --timeout 120 --timeout-method thread > $OUT/pytest_points.log 2>&1
rc=$?; tail -3 $OUT/pytest_points.log; [ $rc -eq 0 ] || { cp $OUT/.orig.so "$LIB"; exit $rc; }
for rep in 1 2; do
  for v in "$@"; do
    cp "$v" "$LIB"
    for args in "--mode fan --width 1920 --height 1080" "--mode fan --width 3840 --height 2160"; do
      timeout -k 10 120 python tools/bench_scene.py $args --frames 400 > $OUT/s.json 2> $OUT/s.err \
        || { tail -5 $OUT/s.err; cp $OUT/.orig.so "$LIB"; exit 1; }
      python -c "
import json,sys; d=json.load(open('$OUT/s.json'))
print('%-20s rep%s %-4s %4dx%-4d ms/frame %.4f' % (sys.argv[1].split('/')[-1], sys.argv[2], d['mode'], d['width'], d['height'], d['ms_per_frame']))
" "$v" "$rep" | tee -a $OUT/scene_ab.txt
    done
  done
done
cp $OUT/.orig.so "$LIB"
