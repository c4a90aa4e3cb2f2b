#!/bin/bash
# Device assembly of geo_render.hip (gfx950, the build's flags) for a git
# revision, or the working tree with REV=.:  bash tools/isa.sh REV OUT.s
set -eu
REV=$1
OUT=$(realpath -m "$2")
ROOT=$(cd "$(dirname "$0")/.." && pwd)
if [ "$REV" = "." ]; then SRC=$ROOT; else
  SRC=$(mktemp -d); trap 'rm -rf "$SRC"' EXIT
  git -C "$ROOT" archive "$REV" schwarzschild_raytracer_wgpu_amd/csrc include __graft_entry__.py | tar -x -C "$SRC"
fi
cd "$SRC/schwarzschild_raytracer_wgpu_amd/csrc"
python3 - "$OUT" <<'PY'
import os, subprocess, sys
sys.path.insert(0, "../..")
import __graft_entry__ as g
flags = [f for f in g.HIP_FLAGS if f not in ("-shared", "-fPIC")]
subprocess.run([g.HIPCC, *flags, "--cuda-device-only", "-S", "-o", sys.argv[1], "geo_render.hip"], check=True)
PY
