#!/bin/bash
# A/B of two prebuilt libgeo.so files on one GPU box (for changes with no
# compile-time switch, e.g. a spec change mirrored in the oracle):
#   BENCH_ARGS="--config cfg5_8k_adaptive --no-cpu-baseline" bash tools/gpu_ab_lib.sh OLD.so NEW.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
cp "$LIB" gpurun_out/.libgeo_orig.so
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    cp "$v" "$LIB"
    timeout -k 10 300 python ${BENCH:-bench.py} ${BENCH_ARGS:---no-cpu-baseline --steps 400} > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab.err; cp gpurun_out/.libgeo_orig.so "$LIB"; exit $rc; }
    python -c "
import json,sys; d=json.load(open('gpurun_out/ab.json'))
print('%-40s rep%s  ms/frame %.4f  kernel avg %.4f  frac %.3f' % (sys.argv[1], sys.argv[2], d['ms_per_step'], d['kernel_ms']['avg'], d['roofline']['frac']))
" "$v" "$rep" | tee -a gpurun_out/ab_summary.txt
  done
done
cp gpurun_out/.libgeo_orig.so "$LIB"
