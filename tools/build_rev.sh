#!/bin/bash
# Build libgeo.so of git revision REV (same sources and flags as that
# revision's __graft_entry__.build()) into OUT, for A/B runs against an
# earlier kernel:  bash tools/build_rev.sh HEAD~1 tools/ubench/libgeo_prev.so
set -eu
REV=$1
OUT=$(realpath -m "$2")
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
git -C "$ROOT" archive "$REV" schwarzschild_raytracer_wgpu_amd/csrc include __graft_entry__.py | tar -x -C "$T"
cd "$T"
python - "$OUT" <<'PY'
import os, subprocess, sys
import __graft_entry__ as g
subprocess.run([g.HIPCC, *g.HIP_FLAGS, "-o", sys.argv[1], *[os.path.join(g.CSRC, s) for s in g.SOURCES]],
               check=True, cwd=g.CSRC)
PY
echo "$OUT"
