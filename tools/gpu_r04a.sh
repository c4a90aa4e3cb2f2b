#!/bin/bash
# Round-4 first session: the new comparator tests, the metric's bench line
# (cpu_baseline.matches_gpu), config 2 on the current tree (bench + rocprofv3
# stats), the fan-mode draw's HBM roofline (bench + stats + PMC passes with
# occupancy), and bench.py's own N-rank launcher as a gloo rehearsal.
#   bash tools/gpu_r04a.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r04a}
step() { echo "== $*"; }

step pytest
GEO_F64_BAR_OUT="$OUT/f64bar_$TAG" timeout -k 10 600 python -u -m pytest tests/test_gpu_cpu_path.py tests/test_gpu_f64_bar.py tests/test_bench.py -x -v --timeout 300 \
    --timeout-method thread > "$OUT/pytest_$TAG.log" 2>&1 || { tail -30 "$OUT/pytest_$TAG.log"; exit 1; }
tail -3 "$OUT/pytest_$TAG.log"

step bench cfg3
timeout -k 10 300 python bench.py > "$OUT/bench_${TAG}_cfg3.json" 2> "$OUT/bench_${TAG}_cfg3.err" || { tail -5 "$OUT/bench_${TAG}_cfg3.err"; exit 1; }
step bench cfg2
timeout -k 10 300 python bench.py --config cfg2_1080p > "$OUT/bench_${TAG}_cfg2.json" 2> "$OUT/bench_${TAG}_cfg2.err" || { tail -5 "$OUT/bench_${TAG}_cfg2.err"; exit 1; }
step bench fan
timeout -k 10 300 python bench.py --mode fan > "$OUT/bench_${TAG}_fan.json" 2> "$OUT/bench_${TAG}_fan.err" || { tail -5 "$OUT/bench_${TAG}_fan.err"; exit 1; }
step launcher gloo 2
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_${TAG}_gloo2.json" 2> "$OUT/bench_${TAG}_gloo2.err" || { tail -5 "$OUT/bench_${TAG}_gloo2.err"; exit 1; }

cd /tmp && export TMPDIR=/tmp
step rocprof cfg2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_cfg2" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline --config cfg2_1080p > "$OUT/prof_${TAG}_cfg2.log" 2>&1 || exit 1
step rocprof fan
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_fan" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline --mode fan > "$OUT/prof_${TAG}_fan.log" 2>&1 || exit 1
cd "$ROOT"
step pmc fan
CONFIG=cfg3_4k EXTRA_ARGS="--mode fan" bash tools/gpu_pmc.sh pmcfan_$TAG \
    "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
    "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
    "GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES MeanOccupancyPerCU" "TCC_HIT_sum TCC_MISS_sum" || exit 1
python tools/pmc_to_profile.py pmcfan_$TAG "$OUT/${TAG}_cfg3_4k_fan_pmc.json" "cfg3_4k (3840x2160, fan)" \
    "geo_render_kernel<1, 0, false>" > /dev/null || exit 1
echo ok
