#!/bin/bash
# tools/bench_points.py at several warm-up lengths (clock ramp check).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in "$@"; do
  timeout -k 10 200 python tools/bench_points.py --warmup $w --cpu-connectors 200 > gpurun_out/bp.json 2>gpurun_out/bp.err || exit $?
  python -c "
import json,sys; d=json.load(open('gpurun_out/bp.json'))
print('warmup', sys.argv[1], 'ms/step %.4f' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'], 'achieved', d['roofline']['achieved'])
" $w
done
