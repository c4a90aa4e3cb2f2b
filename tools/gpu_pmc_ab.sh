#!/bin/bash
# One PMC pass per compile-time variant of libgeo (same counters), to compare
# cycles, VALU activity and the effective clock of two builds.
#   bash tools/gpu_pmc_ab.sh "COUNTERS" "-DX=0" "-DX=1"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmcab; mkdir -p "$OUT"
CTRS=$1; shift
i=0
for v in "$@"; do
  i=$((i+1))
  python -c "
import sys, subprocess, __graft_entry__ as g
cmd = [g.HIPCC, *g.HIP_FLAGS, *sys.argv[1].split(), '-o', g.LIB, *[g.os.path.join(g.CSRC, s) for s in g.SOURCES]]
subprocess.run(cmd, check=True, cwd=g.CSRC)
" "$v" || exit 1
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d "$OUT/v$i" -o run \
     -- python3 "$ROOT/bench.py" --steps 40 --warmup 5 --spinup-frames 300 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/v$i.log" 2>&1) || { tail -5 "$OUT/v$i.log"; exit 1; }
  echo "variant $i: $v"
  python - "$OUT/v$i" <<'PY'
import glob, sys
sys.path.insert(0, "tools")
from pmc_summary import load
files = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)
c, d = load(files[0], kernel="geo_render")
dur = sum(d.values()) / len(d)
for k, v in sorted(c.items()):
    print(f"  {k:26s} {v:,.1f}")
print(f"  {'dispatch_ns':26s} {dur:,.1f}")
if "GRBM_GUI_ACTIVE" in c:
    print(f"  {'clock_GHz':26s} {c['GRBM_GUI_ACTIVE'] / 8 / dur:.3f}")
PY
done
