#!/bin/bash
# A/B of compile-time variants of libgeo on the GPU box: builds each variant
# (extra hipcc flags) in place and runs the default bench, twice, interleaved.
#   bash tools/gpu_ab.sh "-DGEO_GROUP_UNROLL=1" "-DGEO_GROUP_UNROLL=2"
#   BENCH=tools/bench_points.py BENCH_ARGS="--cpu-connectors 200" bash tools/gpu_ab.sh "-DX=0" "-DX=1"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    python -c "
import sys, subprocess, __graft_entry__ as g
cmd = [g.HIPCC, *g.HIP_FLAGS, *sys.argv[1].split(), '-o', g.LIB, *[g.os.path.join(g.CSRC, s) for s in g.SOURCES]]
subprocess.run(cmd, check=True, cwd=g.CSRC)
" "$v" || exit 1
    timeout -k 10 300 python ${BENCH:-bench.py} ${BENCH_ARGS:---no-cpu-baseline --steps 400} > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab.err; exit $rc; }
    python -c "
import json,sys; d=json.load(open('gpurun_out/ab.json'))
print('%-28s rep%s  ms/frame %.4f  kernel avg %.4f  frac %.3f' % (sys.argv[1], sys.argv[2], d['ms_per_step'], d['kernel_ms']['avg'], d['roofline']['frac']))
" "$v" "$rep" | tee -a gpurun_out/ab_summary.txt
  done
done
