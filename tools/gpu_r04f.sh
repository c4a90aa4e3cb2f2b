#!/bin/bash
# Round-4 session f: the GPU suite, fan-mode and config-2 bench lines (with the
# CPU comparator), config 5's PMC passes, the fan draw's rocprofv3 trace, and
# the N-rank host-bound probe with the learned dispatch order.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r04f}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_$TAG.log" 2>&1 || { tail -30 "$OUT/pytest_$TAG.log"; exit 1; }
tail -1 "$OUT/pytest_$TAG.log"
for M in "--mode fan" "--config cfg2_1080p"; do
  N=$(echo $M | tr -d ' -' )
  timeout -k 10 300 python bench.py $M > "$OUT/bench_${TAG}_$N.json" 2> "$OUT/bench_${TAG}_$N.err" || { tail -5 "$OUT/bench_${TAG}_$N.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_${TAG}_$N.json')); r=d['roofline']; print('$N', round(d['ms_per_step'],5), round(d['kernel_ms']['avg'],5), r['bound'], round(r['frac'],4), d['cpu_baseline']['matches_gpu']['ok'])"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_fan" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline --mode fan > "$OUT/prof_${TAG}_fan.log" 2>&1) || exit 1
python tools/trace_window.py "$OUT/prof_${TAG}_fan/run_kernel_trace.csv" --kernel "geo_render_kernel<1, 0, false>" | tail -3
SETS=("GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
      "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FLOPS_FP32"
      "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES MeanOccupancyPerCU")
CONFIG=cfg5_8k_adaptive bash tools/gpu_pmc.sh pmc5_$TAG "${SETS[@]}" || exit 1
python tools/pmc_to_profile.py pmc5_$TAG "$OUT/${TAG}_cfg5_8k_adaptive_pmc.json" "cfg5_8k_adaptive (7680x4320, RK5(4) tol 1e-6, adaptive)" "geo_render_kernel<GEO_MODE_ADAPTIVE, kCurvedOut>" || exit 1
for A in "8 1 8 2" "8 2 8 2" "4 1 8 2"; do
  timeout -k 10 200 python tools/host_bound_probe.py $A > "$OUT/hostprobe_${TAG}_${A// /_}.txt" 2>&1 || exit 1
  echo "== host probe $A"; tail -4 "$OUT/hostprobe_${TAG}_${A// /_}.txt"
done
echo ok
