"""Turn rocprofv3 --pmc passes (tools/gpu_pmc.sh) into a committed profile
summary under profiles/: per-dispatch counter means for geo_render_kernel and
the derived numbers bench.py and DESIGN.md quote.

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are L2
memory-side (fabric) request bytes (Infinity-Cache hits included); the 2x
FETCH correction applies to 16-B/lane streaming reads only, and this kernel's
reads are 4-B texel gathers, so FETCH_SIZE is used as is (uncalibrated width).
"""
import json
import sys

sys.path.insert(0, "tools")
from pmc_summary import load  # noqa: E402
import glob  # noqa: E402

tag, out, workload = sys.argv[1], sys.argv[2], sys.argv[3]
c = {}
dur = {}
for p in sorted(sum((glob.glob(f"gpurun_out/{t}_*/run_counter_collection.csv") for t in tag.split(",")), [])):
    cc, d = load(p)
    c.update(cc)
    dur.update(d)
dur_ns = sum(dur.values()) / len(dur)
xcd_cycles = c["GRBM_GUI_ACTIVE"] / 8.0
res = {
    "kernel": sys.argv[4] if len(sys.argv) > 4 else "geo_render_kernel<GEO_MODE_DIRECT, kCurvedOut>",
    "workload": workload,
    "source": f"rocprofv3 --kernel-trace --pmc (separate passes), gpurun_out/{tag}_*",
    "counters_per_dispatch": c,
    "dispatch_ns_profiled": dur_ns,
    "derived": {
        "clock_ghz": xcd_cycles / dur_ns,
        "valu_issue_utilisation": c["SQ_INSTS_VALU"] * 2.0 / 1024.0 / xcd_cycles,
        "valu_per_simd_cycle": c["SQ_INSTS_VALU"] / 1024.0 / xcd_cycles,
        "salu_per_cu_cycle": c["SQ_INSTS_SALU"] / 256.0 / xcd_cycles,
        "lane_utilisation": c.get("SQ_THREAD_CYCLES_VALU", 0) / (64.0 * c["SQ_INSTS_VALU"]),
        "hw_fp32_flops": c.get("SQ_INSTS_VALU_FLOPS_FP32", 0) * 64.0,
        "hw_fp32_tflops": c.get("SQ_INSTS_VALU_FLOPS_FP32", 0) * 64.0 / dur_ns / 1e3,
        "hbm_read_bytes": c["FETCH_SIZE"] * 1024.0,
        "hbm_write_bytes": c["WRITE_SIZE"] * 1024.0,
        "traffic_bytes": (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0,
    },
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["derived"], indent=1))
