#!/bin/bash
# Session r04k, the round-4 evidence set on the final tree: GPU suite, smoke,
# bench lines (config 3 = the metric, configs 2 and 5, the fan draw; the
# frame-pipelined figures beside them), rocprofv3 kernel stats and timed
# windows for each, PMC passes for each, a long fuzz sweep, gloo rehearsals.
#   PART=1 bash tools/gpu_r04k.sh [TAG]   (suite, smoke, bench lines, rocprofv3)
#   PART=2 bash tools/gpu_r04k.sh [TAG]   (PMC passes, fuzz sweep, gloo rehearsals)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r04k}
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_$TAG.log" 2>&1 || { tail -30 "$OUT/pytest_$TAG.log"; exit 1; }
tail -1 "$OUT/pytest_$TAG.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { tail -5 "$OUT/smoke_$TAG.log"; exit 1; }
tail -1 "$OUT/smoke_$TAG.log"
declare -A ARGS=([cfg3_4k]="" [cfg2_1080p]="--config cfg2_1080p" [cfg5_8k_adaptive]="--config cfg5_8k_adaptive"
                 [cfg3_4k_fan]="--mode fan")
declare -A KERN=([cfg3_4k]="geo_render_kernel<0, 0, false, 1u>" [cfg2_1080p]="geo_render_kernel<0, 0, false, 1u>"
                 [cfg5_8k_adaptive]="geo_render_kernel<2, 0, false, 1u>" [cfg3_4k_fan]="geo_render_kernel<1, 0, false, 1u>")
for C in cfg3_4k cfg2_1080p cfg5_8k_adaptive cfg3_4k_fan; do
  timeout -k 10 400 python bench.py ${ARGS[$C]} --pipelined > "$OUT/bench_${TAG}_$C.json" 2> "$OUT/bench_${TAG}_$C.err" \
      || { tail -5 "$OUT/bench_${TAG}_$C.err"; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_${TAG}_$C.json')); r=d['roofline']; p=d['pipelined']
print('$C', 'ms/step %.5f' % d['ms_per_step'], 'kernel %.5f' % d['kernel_ms']['avg'], r['bound'], 'frac %.4f' % r['frac'],
      'pipelined ms/step %.5f' % p['ms_per_step'], 'cpu %.3g' % d['cpu_baseline']['value'], d['cpu_baseline']['matches_gpu']['ok'])"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_$C" -o run \
      -- python3 "$ROOT/bench.py" ${ARGS[$C]} --no-cpu-baseline > "$OUT/prof_${TAG}_$C.log" 2>&1) || { tail -5 "$OUT/prof_${TAG}_$C.log"; exit 1; }
  python tools/trace_window.py "$OUT/prof_${TAG}_$C/run_kernel_trace.csv" --kernel "${KERN[$C]}" > "$OUT/${TAG}_${C}_trace_window.txt" || exit 1
  tail -1 "$OUT/${TAG}_${C}_trace_window.txt"
done
exit 0
fi
SETS=("GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
      "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FLOPS_FP32"
      "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES MeanOccupancyPerCU")
CONFIG=cfg3_4k bash tools/gpu_pmc.sh pmc3_$TAG "${SETS[@]}" || exit 1
python tools/pmc_to_profile.py pmc3_$TAG "$OUT/${TAG}_cfg3_4k_pmc.json" "cfg3_4k (3840x2160, 2048 steps, direct)" > /dev/null || exit 1
CONFIG=cfg2_1080p bash tools/gpu_pmc.sh pmc2_$TAG "${SETS[@]}" || exit 1
python tools/pmc_to_profile.py pmc2_$TAG "$OUT/${TAG}_cfg2_1080p_pmc.json" "cfg2_1080p (1920x1080, 512 steps, direct)" > /dev/null || exit 1
CONFIG=cfg3_4k EXTRA_ARGS="--mode fan" bash tools/gpu_pmc.sh pmcf_$TAG "${SETS[@]}" || exit 1
python tools/pmc_to_profile.py pmcf_$TAG "$OUT/${TAG}_cfg3_4k_fan_pmc.json" "cfg3_4k (3840x2160, fan)" "geo_render_kernel<GEO_MODE_FAN> (two pixels per lane)" > /dev/null || exit 1
CONFIG=cfg5_8k_adaptive bash tools/gpu_pmc.sh pmc5_$TAG "${SETS[@]}" || exit 1
python tools/pmc_to_profile.py pmc5_$TAG "$OUT/${TAG}_cfg5_8k_adaptive_pmc.json" "cfg5_8k_adaptive (7680x4320, RK5(4) tol 1e-6, adaptive)" "geo_render_kernel<GEO_MODE_ADAPTIVE, kCurvedOut>" > /dev/null || exit 1
N=${FUZZ_N:-20000} BASE=${FUZZ_BASE:-400000} bash tools/gpu_fuzz_sweep.sh > "$OUT/${TAG}_fuzz_sweep.txt" 2>&1 || { tail -5 "$OUT/${TAG}_fuzz_sweep.txt"; exit 1; }
grep fuzz "$OUT/${TAG}_fuzz_sweep.txt"
TAG=$TAG bash tools/gpu_dist_rehearse.sh > "$OUT/${TAG}_dist_rehearse.txt" 2>&1 || { tail -5 "$OUT/${TAG}_dist_rehearse.txt"; exit 1; }
grep -c "frame-check" "$OUT/${TAG}_dist_rehearse.txt"
echo ok
