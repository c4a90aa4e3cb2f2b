#!/bin/bash
# Session r04m: the whole GPU suite and smoke on the final tree, then the
# driver's bench form (N = 1, 20 steps) and the default 200-step line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/r04m_gpu_suite.txt 2>&1 || { tail -30 $OUT/r04m_gpu_suite.txt; exit 1; }
tail -1 $OUT/r04m_gpu_suite.txt
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r04m_smoke.txt 2>&1 || { tail -5 $OUT/r04m_smoke.txt; exit 1; }
tail -1 $OUT/r04m_smoke.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r04m_bench_driver_form.json 2> $OUT/r04m_bench_driver_form.err \
  || { tail -5 $OUT/r04m_bench_driver_form.err; exit 1; }
timeout -k 10 300 python3 bench.py > $OUT/r04m_bench_default.json 2> $OUT/r04m_bench_default.err \
  || { tail -5 $OUT/r04m_bench_default.err; exit 1; }
for f in driver_form default; do python -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']
print(sys.argv[2], 'value %.4g' % d['value'], 'ms/step %.5f' % d['ms_per_step'], 'kernel %.5f' % d['kernel_ms']['avg'], 'frac %.4f' % r['frac'], 'timed', d['kernel_ms']['frames_timed'], 'cpu ok', d['cpu_baseline']['matches_gpu']['ok'])" $OUT/r04m_bench_$f.json $f; done
