"""Average duration of the render kernel over bench.py's timed region, from a
rocprofv3 --kernel-trace CSV of `bench.py` (N = 1, one render stream).

bench.py launches the render kernel in this order: 1 diagnostic frame, the
clock spin-up (--spinup-frames), the warmup, the K timed frames, then the K
compute-only frames.  rocprofv3's --stats average covers all of them (the
spin-up frames run while the clock ramps); this prints the average over the
timed window beside it, the figure bench.py's in-region HIP events estimate.

    python tools/trace_window.py gpurun_out/prof_r02g/run_kernel_trace.csv [--spinup 300 --warmup 20 --steps 200]
"""
import argparse
import csv
import statistics


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--kernel", default="geo_render_kernel<0, 0, false, 1u>")
    p.add_argument("--spinup", type=int, default=300)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--steps", type=int, default=200)
    a = p.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
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
    print(f"spin-up frames     avg {statistics.fmean(sp):.4f} ms (first 20: {statistics.fmean(sp[:20]):.4f} ms)")


if __name__ == "__main__":
    main()
