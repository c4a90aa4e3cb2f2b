#!/bin/bash
# The driver's bench command (--steps 20 --warmup 5) back to back with the
# long form, to compare the two on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/short; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/s20_$i.json 2> $OUT/s20_$i.err || exit $?
  python -c "import json;d=json.load(open('$OUT/s20_$i.json'));print('s20',d['ms_per_step'],d['kernel_ms'],d['roofline']['frac'])"
done
timeout -k 10 200 python bench.py --gpus 1 --no-cpu-baseline > $OUT/s200.json 2> $OUT/s200.err || exit $?
python -c "import json;d=json.load(open('$OUT/s200.json'));print('s200',d['ms_per_step'],d['kernel_ms'],d['roofline']['frac'])"
