"""Average duration of the render kernel over bench.py's timed region, from a
rocprofv3 --kernel-trace CSV of `bench.py` (N = 1, one render stream).

bench.py launches the render kernel in this order: 1 diagnostic frame, the
clock spin-up (--spinup-frames), the warmup, the K timed frames, then the K
compute-only frames.  rocprofv3's --stats average covers all of them (the
spin-up frames run while the clock ramps); this prints the average over the
timed window beside it, the figure bench.py's in-region HIP events estimate.

With --bench (the bench line of the SAME invocation, run under rocprofv3),
the window is taken from the line (spinup_frames, warmup, steps), the kernel
from its roofline (geo_render_kernel<MODE, ...>: the instantiation with the
most launches), and the roofline fraction is recomputed from the trace:
algorithmic flops (or bytes) per launch / the window's average launch time /
peak, against the line's own `roofline.frac` (north star: they agree within
1 %).

    python tools/trace_window.py TRACE.csv [--spinup 300 --warmup 20 --steps 200]
    python tools/trace_window.py TRACE.csv --bench BENCH.json [--json OUT.json]
"""
import argparse
import collections
import csv
import json
import statistics


def bench_line(path):
    with open(path) as f:
        lines = [ln for ln in f.read().splitlines() if ln.lstrip().startswith("{")]
    if not lines:
        raise SystemExit(f"{path}: no JSON line")
    return json.loads(lines[-1])


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--kernel", default="geo_render_kernel<0, 0, false, 1u>")
    p.add_argument("--spinup", type=int, default=300)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--bench", default=None, help="the bench line of the traced invocation")
    p.add_argument("--json", default=None, help="write the comparison here")
    a = p.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    line = None
    if a.bench:
        line = bench_line(a.bench)
        a.spinup, a.warmup, a.steps = line["spinup_frames"], line["warmup"], line["steps"]
        mode = line["roofline"]["kernel"].split("<", 1)[1].split(">", 1)[0].split(",")[0].strip()
        names = collections.Counter(r["Kernel_Name"] for r in rows
                                    if f"geo_render_kernel<{mode}," in r["Kernel_Name"])
        if not names:
            raise SystemExit(f"no geo_render_kernel<{mode}, ...> launches in {a.trace}")
        a.kernel = names.most_common(1)[0][0]
    rows = [r for r in rows if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]  # ms
    t0 = 1 + a.spinup + a.warmup
    win = dur[t0:t0 + a.steps]
    if len(win) != a.steps:
        raise SystemExit(f"{len(dur)} launches of {a.kernel}: no full timed window at {t0}..{t0 + a.steps}")
    print(f"kernel {a.kernel}: {len(dur)} launches")
    print(f"all launches       avg {statistics.fmean(dur):.4f} ms  median {statistics.median(dur):.4f} ms")
    print(f"timed window [{t0}, {t0 + a.steps}) avg {statistics.fmean(win):.4f} ms  median {statistics.median(win):.4f} ms")
    sp = dur[1:1 + a.spinup]
    if sp:
        print(f"spin-up frames     avg {statistics.fmean(sp):.4f} ms (first 20: {statistics.fmean(sp[:20]):.4f} ms)")
    if line is None:
        return
    rf = line["roofline"]
    work = rf.get("algorithmic_flops_per_launch") or rf.get("algorithmic_bytes_per_launch")
    scale = 1e12 if rf["unit"] == "TFLOP/s" else 1e9
    win_ms = statistics.fmean(win)
    frac_trace = work / (win_ms * 1e-3) / scale / rf["peak"]
    out = {"kernel": a.kernel, "launches": len(dur), "window": [t0, t0 + a.steps],
           "window_avg_ms": win_ms, "window_median_ms": statistics.median(win),
           "all_launches_avg_ms": statistics.fmean(dur),
           "line_kernel_ms_avg": line["kernel_ms"]["avg"], "line_frac": rf["frac"], "trace_frac": frac_trace,
           "trace_over_line": frac_trace / rf["frac"], "work_per_launch": work, "unit": rf["unit"],
           "peak": rf["peak"], "line_value": line["value"], "workload": line["config"]["workload"],
           "n_gpus": line["n_gpus"], "source": a.trace.split("gpurun_out/")[-1]}
    print(f"roofline: line frac {rf['frac']:.4f} (events avg {line['kernel_ms']['avg']:.4f} ms), trace frac "
          f"{frac_trace:.4f} (window avg {win_ms:.4f} ms): trace/line {frac_trace / rf['frac']:.4f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
