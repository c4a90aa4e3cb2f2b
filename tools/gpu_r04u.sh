#!/bin/bash
# Round 4 (u): the accretion-disk update in one launch (orbit step, respawn
# reset and update_ray fused) and the two point meshes drawn in one launch.
# The points GPU tests on the new library, then the reference's whole frame
# (tools/bench_scene.py, fan and direct mode) A/B against the previous library,
# interleaved, then a kernel trace of the new fan-mode frame.
#   bash tools/gpu_r04u.sh OLD.so NEW.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04u
mkdir -p $OUT
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
OLD=$1
NEW=$2
cp "$NEW" "$LIB"
timeout -k 10 300 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_parity.py -m gpu -x -q -k "point or disk or ray" \
  --timeout 120 --timeout-method thread > $OUT/pytest_points.log 2>&1
rc=$?; tail -3 $OUT/pytest_points.log; [ $rc -eq 0 ] || exit $rc
# the same disk run (orbits, respawns, both meshes drawn) on both libraries: byte for byte
timeout -k 10 120 python tools/points_dump.py $OUT/points_new.npz || exit $?
cp "$OLD" "$LIB"
timeout -k 10 120 python tools/points_dump.py $OUT/points_old.npz; rc=$?
cp "$NEW" "$LIB"; [ $rc -eq 0 ] || exit $rc
python -c "
import numpy as np; a = np.load('$OUT/points_old.npz'); b = np.load('$OUT/points_new.npz')
bad = [k for k in a.files if a[k].tobytes() != b[k].tobytes()]
print('points state old vs new:', 'identical' if not bad else 'DIFFER in %s' % bad, '(%d arrays)' % len(a.files))
raise SystemExit(1 if bad else 0)
" | tee $OUT/points_ab.txt || exit 1
: > $OUT/scene_ab.txt
for rep in 1 2 3; do
  for v in "$OLD" "$NEW"; do
    cp "$v" "$LIB"
    for args in "--mode fan --width 1920 --height 1080" "--mode fan --width 3840 --height 2160" \
                "--mode direct --width 3840 --height 2160"; do
      timeout -k 10 120 python tools/bench_scene.py $args --frames 400 > $OUT/s.json 2> $OUT/s.err
      rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/s.err; cp "$NEW" "$LIB"; exit $rc; }
      python -c "
import json,sys; d=json.load(open('$OUT/s.json'))
print('%-28s rep%s %-6s %4dx%-4d ms/frame %.4f  parts %s' % (sys.argv[1].split('/')[-1], sys.argv[2], d['mode'], d['width'], d['height'], d['ms_per_frame'], {k: round(v, 4) for k, v in d['gpu_ms'].items()}))
" "$v" "$rep" | tee -a $OUT/scene_ab.txt
    done
  done
done
cp "$NEW" "$LIB"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o scene -- python3 tools/bench_scene.py --mode fan \
  --width 1920 --height 1080 --frames 300 > $OUT/scene_fan_1080_traced.json 2> $OUT/prof.err
