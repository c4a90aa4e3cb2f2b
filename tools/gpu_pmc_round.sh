#!/bin/bash
# Round PMC session: rocprofv3 --pmc passes (each its own run, kernel trace
# only) for the config-3 and config-5 render kernels, and the op_rates
# microbenchmark under the same issue counters (its v_fma_f32 streams give the
# VALU issue ceiling in wave-instructions per SIMD-cycle).
#   bash tools/gpu_pmc_round.sh r02
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-r02}
mkdir -p gpurun_out
SETS=("GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
      "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FLOPS_FP32"
      "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum")
CONFIG=cfg3_4k bash tools/gpu_pmc.sh pmc3_$TAG "${SETS[@]}" || exit $?
CONFIG=cfg5_8k_adaptive bash tools/gpu_pmc.sh pmc5_$TAG "${SETS[@]}" || exit $?
python tools/pmc_to_profile.py pmc3_$TAG gpurun_out/${TAG}_cfg3_4k_pmc.json "cfg3_4k (3840x2160, 2048 steps, direct)" || exit 1
python tools/pmc_to_profile.py pmc5_$TAG gpurun_out/${TAG}_cfg5_8k_adaptive_pmc.json "cfg5_8k_adaptive (7680x4320, RK5(4) tol 1e-6, adaptive)" "geo_render_kernel<GEO_MODE_ADAPTIVE, kCurvedOut>" || exit 1
hipcc --offload-arch=gfx950 -O3 -o /tmp/op_rates tools/ubench/op_rates.hip 2>/dev/null || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES \
    --output-format csv -d "$ROOT/gpurun_out/opr_$TAG" -o run -- /tmp/op_rates > "$ROOT/gpurun_out/opr_$TAG.log" 2>&1) || exit 1
python - "$ROOT/gpurun_out/opr_$TAG" <<'PY'
import collections, csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
name = {}
for r in csv.DictReader(open(f)):
    agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    name[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
best = {}
for d, c in agg.items():
    if c.get("GRBM_GUI_ACTIVE", 0) <= 0:
        continue
    rate = c["SQ_INSTS_VALU"] / 1024.0 / (c["GRBM_GUI_ACTIVE"] / 8.0)
    best[name[d]] = max(best.get(name[d], 0.0), rate)
for k, v in sorted(best.items(), key=lambda kv: -kv[1]):
    print(f"{k:40s} {v:.3f} VALU wave-instr per SIMD-cycle")
PY
