#!/bin/bash
# The one GPU evidence script (replaces the per-session tools/gpu_r0*.sh).
# Every step runs under its own time limit; the first failing step ends the
# call (no retries).  Output goes to gpurun_out/<TAG>/.
#
#   bash tools/evidence.sh TAG STEP [STEP ...]
#
# STEPs:
#   suite            pytest -m gpu (one process) + smoke()
#   tests:<k-expr>   pytest -m gpu -k <k-expr>
#   gloo8 | gloo:N   the driver's N-rank form (N = 8 for gloo8) on this one GPU with gloo:
#                    bench.py --gpus 8 --dist-backend gloo --steps 20 --warmup 5
#                    (self-launcher, --rank0-lead auto, batched launches,
#                    frame_check), its wall time recorded
#   bench:<cfg>[:<mode>[:<steps>]]
#                    bench.py under rocprofv3 --kernel-trace --stats, the
#                    bench line and the trace's timed-window average from the
#                    SAME invocation (tools/trace_window.py)
#   plain:<cfg>[:<mode>[:<steps>]]   bench.py alone (default flags)
#                    (bench and plain: BENCH_ARGS="..." adds bench.py flags, e.g. --ring-f64)
#   pmc:<cfg>[:<mode>]  the PMC passes (each its own rocprofv3 run)
#   motion           bench.py --motion none|orbit|fall x --dispatch learned|natural, N = 1 and --share 1/8
#   timeline[:cases] tools/wave_timeline.py: every wave's span in a launch (diagnostic build)
#   ab:<cfgs>[:reps] interleaved A/B of LIBS="a.so b.so" and/or ABARGS="args;args" (bench lines;
#                    configs comma-separated; replaces the round-5 fpl_ab.sh / batch_ab.sh)
#   fuzz[:n[:base]]  long GPU fuzz sweeps (direct, adversarial, fan, mips, batched launches, ring f64) on new seeds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

heartbeat() {  # keeps gpurun's 3-minute silence watchdog informed during long quiet steps
  (while sleep 30; do date +%T >> "$OUT/heartbeat.txt"; done) &
  HB=$!
}
stop_heartbeat() { kill $HB 2>/dev/null; wait $HB 2>/dev/null; }

for step in "$@"; do
  IFS=: read -r kind a1 a2 a3 <<< "$step"
  echo "== $step ($(date +%T))"
  case $kind in
    suite)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$OUT/gpu_suite.txt" 2>&1
      rc=$?; tail -3 "$OUT/gpu_suite.txt"; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
      rc=$?; tail -1 "$OUT/smoke.txt"; [ $rc -eq 0 ] || exit $rc ;;
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$a1" \
        > "$OUT/tests_${a1//[^A-Za-z0-9_]/_}.txt" 2>&1
      rc=$?; tail -3 "$OUT/tests_${a1//[^A-Za-z0-9_]/_}.txt"; [ $rc -eq 0 ] || exit $rc ;;
    gloo8|gloo)
      # the driver's N-rank form on this one GPU with gloo (gloo8 = gloo:8)
      n=${a1:-8}; [ $kind = gloo8 ] && n=8
      heartbeat
      t0=$(date +%s.%N)
      timeout -k 10 1000 python3 bench.py --gpus $n --dist-backend gloo --steps 20 --warmup 5 \
        > "$OUT/gloo${n}_bench.json" 2> "$OUT/gloo${n}_bench.err"
      rc=$?
      t1=$(date +%s.%N)
      stop_heartbeat
      python3 - "$OUT" "$t0" "$t1" "$rc" "$n" <<'EOF'
import json, sys
out, t0, t1, rc, n = sys.argv[1], float(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
rec = {"cmd": f"python3 bench.py --gpus {n} --dist-backend gloo --steps 20 --warmup 5", "rc": rc,
       "wall_s": round(t1 - t0, 2), "driver_timeout_s": 600}
try:
    d = json.loads(open(f"{out}/gloo{n}_bench.json").read().strip().splitlines()[-1])
    rec.update({k: d[k] for k in ("n_gpus", "world_size", "dist_backend", "value", "ms_per_step", "frame_check")})
    rec["config"] = d["config"]
    rec["per_rank"] = d["per_rank"]
except Exception as e:  # noqa: BLE001
    rec["parse_error"] = repr(e)
json.dump(rec, open(f"{out}/gloo{n}_summary.json", "w"), indent=1)
print(json.dumps({k: rec.get(k) for k in ("rc", "wall_s", "frame_check")}))
EOF
      [ $rc -eq 0 ] || { tail -20 "$OUT/gloo${n}_bench.err"; exit $rc; } ;;
    bench|plain)
      cfg=${a1:-cfg3_4k}; mode=${a2:-}; steps=${a3:-20}
      margs="--config $cfg --steps $steps --warmup 5 ${BENCH_ARGS:-}"; [ -n "$mode" ] && margs="$margs --mode $mode"
      name=${cfg}${mode:+_$mode}
      if [ $kind = plain ]; then
        timeout -k 10 400 python3 bench.py $margs > "$OUT/${name}_bench.json" 2> "$OUT/${name}_bench.err"
        rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/${name}_bench.err"; exit $rc; }
        continue
      fi
      ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" \
          -o run -- python3 "$ROOT/bench.py" $margs > "$OUT/${name}_bench.json" 2> "$OUT/${name}_bench.err" )
      rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/${name}_bench.err"; exit $rc; }
      tr=$(find "$OUT/prof_$name" -name 'run_kernel_trace.csv' | head -n 1)
      st=$(find "$OUT/prof_$name" -name 'run_kernel_stats.csv' | head -n 1)
      cp "$st" "$OUT/${name}_kernel_stats.csv"
      python3 tools/trace_window.py "$tr" --bench "$OUT/${name}_bench.json" --json "$OUT/${name}_trace_window.json" > "$OUT/${name}_trace_window.txt"
      rc=$?; cat "$OUT/${name}_trace_window.txt"; [ $rc -eq 0 ] || exit $rc
      rm -rf "$OUT/prof_$name" ;;
    pmc)
      cfg=${a1:-cfg3_4k}; mode=${a2:-}
      name=${cfg}${mode:+_$mode}
      # the round-4 sets (tools/gpu_pmc.sh limits: <= 8 SQ, 4 TCC, 2 GRBM per pass)
      SETS=("GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
            "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FLOPS_FP32"
            "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
            "GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES MeanOccupancyPerCU")
      EXTRA_ARGS=${mode:+--mode $mode} CONFIG=$cfg bash tools/gpu_pmc.sh "$TAG/pmc_$name" "${SETS[@]}" || exit $?
      # the labels bench.py's pmc_profile() matches: "<cfg> (WxH, ..., <mode>)"
      labels=$(python3 - "$cfg" "$mode" <<'PY'
import sys
from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS
cfg, mode = sys.argv[1], sys.argv[2]
c = CONFIGS[cfg]
m = mode or c.mode
what = {"direct": f"{c.max_steps} steps", "adaptive": f"RK5(4) tol {c.tol:g}", "fan": None}[m]
print(f"{cfg} ({c.width}x{c.height}{', ' + what if what else ''}, {m})")
print({"direct": "geo_render_kernel<GEO_MODE_DIRECT, kCurvedOut>",
       "adaptive": "geo_render_kernel<GEO_MODE_ADAPTIVE, kCurvedOut>",
       "fan": "geo_render_kernel<GEO_MODE_FAN> (two pixels per lane)"}[m])
PY
) || exit $?
      python3 tools/pmc_to_profile.py "$TAG/pmc_$name" "$OUT/${name}_pmc.json" "$(sed -n 1p <<< "$labels")" \
        "$(sed -n 2p <<< "$labels")" > /dev/null || exit $? ;;
    motion)
      # learned vs natural dispatch order on moving frames: N = 1 (one launch
      # per frame) and one 8-rank share alone in batched launches of 8 frames
      # (K distinct uniforms share one learned order); 3 interleaved reps
      : > "$OUT/motion_runs.txt"
      for rep in 1 2 3; do
        for shr in none 1/8; do
          for mot in none orbit fall; do
            for disp in learned natural; do
              sargs=""; [ $shr != none ] && sargs="--share $shr --frames-per-gather 8 --batch-launch on"
              f="$OUT/motion_${mot}_${disp}_${shr/\//of}_$rep.json"
              timeout -k 10 200 python3 bench.py --motion $mot --dispatch $disp --steps 200 --warmup 20 \
                --no-cpu-baseline $sargs > "$f" 2> "$f.err"
              rc=$?; [ $rc -eq 0 ] || { tail -5 "$f.err"; exit $rc; }
              echo "$rep $shr $mot $disp $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms']['avg'], d['value'])" "$f")" \
                | tee -a "$OUT/motion_runs.txt"
            done
          done
        done
      done ;;
    ab)
      # interleaved A/B on one box: ab:<cfg>[,<cfg>...][:reps]; a cfg ending
      # in _fan runs --mode fan.  LIBS="a.so b.so ..." (prebuilt libraries,
      # e.g. from tools/build_variant.py or tools/build_rev.sh; the in-tree
      # library is restored after) and/or ABARGS="args;args;..." (bench.py
      # argument sets, e.g. "--frames-per-launch 1;--frames-per-launch 8" or
      # "--share 1/8 --frames-per-gather 8 --batch-launch on"); each
      # (cfg, args, lib) is one line per rep
      cfgs=${a1:-cfg3_4k}; reps=${a2:-3}
      LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
      cp "$LIB" "$OUT/.orig.so"
      libs=${LIBS:-$OUT/.orig.so}
      IFS=';' read -r -a argsets <<< "${ABARGS:-}"; [ ${#argsets[@]} -eq 0 ] && argsets=("")
      : > "$OUT/ab.txt"
      for rep in $(seq 1 $reps); do
        for c in ${cfgs//,/ }; do
          cargs="--config ${c%_fan}"; [ "$c" != "${c%_fan}" ] && cargs="$cargs --mode fan"
          for xa in "${argsets[@]}"; do
            for v in $libs; do
              cp "$v" "$LIB"
              GEO_AB_VARIANT=1 timeout -k 10 300 python3 bench.py $cargs $xa --no-cpu-baseline --steps 200 > "$OUT/ab.json" 2> "$OUT/ab.err"
              rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/ab.err"; cp "$OUT/.orig.so" "$LIB"; exit $rc; }
              python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1])
r=d.get('ring_f64') or {}
print('%-14s %-44s %-28s rep%s  ms/frame %.5f  kernel %.5f  frac %.4f  frame_check %s  ring %s' % (sys.argv[2], sys.argv[5], sys.argv[3].split('/')[-1], sys.argv[4], d['ms_per_step'], d['kernel_ms']['avg'], d['roofline']['frac'], (d.get('frame_check') or {}).get('ok'), ('%.5f/%.5f %+.4f' % (r['ms_per_step'], r['plain_ms_per_step'], r['overhead'])) if r else '-'))" \
                "$OUT/ab.json" "$c" "$v" "$rep" "${xa:--}" | tee -a "$OUT/ab.txt"
            done
          done
        done
      done
      cp "$OUT/.orig.so" "$LIB" ;;
    fuzz)
      # long GPU fuzz sweeps on seeds beyond the committed ones: fuzz:<n>:<base>
      for t in test_gpu_fuzz_bitexact test_gpu_fuzz_adversarial_bitexact test_gpu_fuzz_fan_mode_bitexact \
               test_gpu_fuzz_mips_bitexact test_gpu_fuzz_batch_bitexact test_ring_fuzz_scenes_against_the_oracle; do
        GEO_FUZZ_N=${a1:-2000} GEO_FUZZ_BASE=${a2:-500000} timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_ring.py \
          -m gpu -q -s -k "$t" --timeout 850 --timeout-method thread > "$OUT/fuzz_$t.txt" 2>&1
        rc=$?; grep -h "^fuzz" "$OUT/fuzz_$t.txt"; tail -1 "$OUT/fuzz_$t.txt"; [ $rc -eq 0 ] || exit $rc
      done ;;
    timeline)
      # per-wave start/end of render launches (diagnostic build, built on the CPU side beforehand:
      # python tools/build_variant.py tools/ab/libgeo_wavelog.so -DGEO_WAVE_LOG=1)
      timeout -k 10 400 python3 tools/wave_timeline.py --out "$OUT/wave_timeline.json" ${a1:+--cases $a1} \
        > "$OUT/wave_timeline.txt" 2> "$OUT/wave_timeline.err"
      rc=$?; cat "$OUT/wave_timeline.txt"; [ $rc -eq 0 ] || { tail -5 "$OUT/wave_timeline.err"; exit $rc; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "evidence $TAG: all steps ok"
