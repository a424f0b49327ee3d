"""Per-hop (or per-launch) medians of rocprofv3 --pmc counters of the step kernel.
Usage: python scripts/pmc_per_hop.py <dir with run_counter_collection.csv> <hops per launch>"""
import csv, glob, statistics, sys, collections
d, hops = sys.argv[1], float(sys.argv[2])
v = collections.defaultdict(list)
for f in glob.glob(d + "/run_counter_collection.csv") + glob.glob(d + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(v):
    x = v[k][1:] or v[k]
    m = statistics.median(x)
    print(f"{k:28s} per launch {m:.4g}  per hop {m / hops:.4g}  (dispatches {len(v[k])})")
