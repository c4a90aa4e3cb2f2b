"""Turn rocprofv3 --pmc passes (tools/gpu_pmc.sh) into a committed profile
summary under profiles/: per-dispatch counter means for geo_render_kernel and
the derived numbers bench.py and DESIGN.md quote.

HBM traffic follows MI355X_MICROARCH.md §HBM: L2 memory-side (fabric)
request bytes, Infinity-Cache hits included.  Reads are counted by request
size, 64 * TCC_EA0_RDREQ_64B + 128 * TCC_EA0_RDREQ_128B: FETCH_SIZE tallies a
128-B request as 64 B on gfx950 (calibrated on a known byte count,
tools/ubench/fetch_calib.hip: a 67.1 MB streaming read reads 33.6 MB of
FETCH_SIZE and exactly 67.1 MB by request size; this kernel's sky gathers
are 99.8 % 128-B requests).  WRITE_SIZE is exact for its 4-B/lane stores (the
same calibration).  A profile without the request counters falls back to
FETCH_SIZE and says so.
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
if "TCC_EA0_RDREQ_128B_sum" in c:
    read_b = 64.0 * c["TCC_EA0_RDREQ_64B_sum"] + 128.0 * c["TCC_EA0_RDREQ_128B_sum"]
    read_src = "64 * TCC_EA0_RDREQ_64B_sum + 128 * TCC_EA0_RDREQ_128B_sum"
else:
    read_b = c["FETCH_SIZE"] * 1024.0
    read_src = "FETCH_SIZE (uncorrected: counts 128-B requests as 64 B)"
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
        "hbm_read_bytes": read_b,
        "hbm_read_source": read_src,
        "hbm_write_bytes": c["WRITE_SIZE"] * 1024.0,
        "traffic_bytes": read_b + c["WRITE_SIZE"] * 1024.0,
    },
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["derived"], indent=1))
