import csv, collections, sys, json
d = sys.argv[1]; events = float(sys.argv[2]) if len(sys.argv) > 2 else None
tot = collections.defaultdict(list)
for p in ["a", "b", "c"]:
    try:
        for r in csv.DictReader(open(f"{d}/{p}/run_counter_collection.csv")):
            if "step_kernel" in r["Kernel_Name"]:
                tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
    except FileNotFoundError:
        pass
for k, v in sorted(tot.items()):
    m = sorted(v)[len(v) // 2]
    print(f"{k:24s} median={m:.4e}" + (f"  per_event={m/events:.1f}" if events else ""))
