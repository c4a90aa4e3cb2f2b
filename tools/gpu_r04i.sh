#!/bin/bash
# Session r04i: a launch's fixed vs per-pixel cost (fan draw and direct
# mode, tools/ubench/size_scaling.py), then a fuzz sweep on new seeds with
# the round-4 library (direct, adversarial, fan, mips).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in fan direct; do
  timeout -k 10 300 python tools/ubench/size_scaling.py $m 100 > gpurun_out/r04i_size_scaling_$m.json 2> gpurun_out/r04i_size_scaling_$m.err \
    || { tail -5 gpurun_out/r04i_size_scaling_$m.err; exit 1; }
  python -c "
import json,sys; d=json.load(open(sys.argv[1])); f=d['fit_kernel_ms_median']
for r in d['sizes']: print('%-7s %5dx%-5d kernel median %.5f ms  wall/launch %.5f ms' % (d['mode'], r['width'], r['height'], r['kernel_ms_median'], r['wall_ms_per_launch']))
print('%-7s fit: %.5f ms + %.5f ms/Mpx (max residual %.5f ms)' % (d['mode'], f['intercept_ms'], f['ms_per_mpixel'], f['residual_max_ms']))
" gpurun_out/r04i_size_scaling_$m.json | tee -a gpurun_out/r04i_size_scaling.txt
done
N=${N:-3000} BASE=${BASE:-300000} bash tools/gpu_fuzz_sweep.sh 2>&1 | tee gpurun_out/r04i_fuzz_sweep.txt
exit ${PIPESTATUS[0]}
