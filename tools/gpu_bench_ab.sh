#!/bin/bash
# A/B of bench.py argument sets on one box, interleaved, twice.
#   bash tools/gpu_bench_ab.sh "--render-streams 1" "--render-streams 2"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline $v > gpurun_out/bab.json 2> gpurun_out/bab.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bab.err; exit $rc; }
    python -c "
import json,sys; d=json.load(open('gpurun_out/bab.json'))
print('%-36s rep%s  ms/frame %.4f  kernel avg %.4f  frac %.3f  value %.4e' % (sys.argv[1], sys.argv[2], d['ms_per_step'], d['kernel_ms']['avg'], d['roofline']['frac'], d['value']))
" "$v" "$rep"
  done
done
