"""Build libgeo.so with extra compiler flags into a given path (A/B variants).

    python tools/build_variant.py OUT.so [-DX=1 -falign-loops=64 ...]

Same sources and flags as __graft_entry__.build(); the in-tree library is
not touched.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

out = os.path.abspath(sys.argv[1])
cmd = [ge.HIPCC, *ge.HIP_FLAGS, *sys.argv[2:], "-o", out, *[os.path.join(ge.CSRC, s) for s in ge.SOURCES]]
subprocess.run(cmd, check=True, cwd=ge.CSRC)
print(out)
