"""Summarise rocprofv3 --pmc CSVs for the render kernel (per dispatch means)."""
import collections
import csv
import glob
import sys


def load(pattern, kernel="geo_render_kernel"):
    per = collections.defaultdict(list)
    dur = []
    for f in sorted(glob.glob(pattern)):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
                dur.append((r["Dispatch_Id"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        for (d, c), v in agg.items():
            per[c].append(v)
    return {c: sum(v) / len(v) for c, v in per.items()}, dict(dur)


if __name__ == "__main__":
    tag = sys.argv[1]
    allc = {}
    for p in sorted(glob.glob(f"gpurun_out/{tag}_*/run_counter_collection.csv")):
        c, d = load(p)
        allc.update(c)
        if d:
            allc.setdefault("_dur_ns", sum(d.values()) / len(d))
    for k, v in sorted(allc.items()):
        print(f"{k:28s} {v:,.1f}")
