"""Turn a profile_round.sh output dir into profiles/<tag>/ summaries + an entry of
profiles/pmc_traffic.json and of profiles/pmc_sq.json (one per profiled workload: topology,
replicas, hops, library build id — bench.py attaches them to its line only for that build).

Issue utilisation (pmc_sq.json), from the SQ passes: GRBM_GUI_ACTIVE sums the 8 XCDs, so one
XCD's active cycles = GRBM_GUI_ACTIVE / 8; salu_busy = SALU instructions / (cycles x 256 CUs)
(one scalar unit per CU, at most one issue per cycle); valu_busy = 2 x VALU instructions /
(cycles x 1024 SIMDs) (a wave64 VALU instruction occupies a SIMD-32 for 2 cycles).

HBM bytes per launch of the step kernel (prisma_step_kernel_t / prisma_mem_step_kernel)
= 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(MI355X_MICROARCH.md 'HBM': FETCH_SIZE counts half the bytes of wide coalesced reads on
gfx950 — our staging reads are 16 B/lane; WRITE_SIZE is exact for 16-B stores, our
record stores are 4-8 B and are reported as measured, uncalibrated).
"""
import csv, json, os, shutil, statistics, sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles", tag)
os.makedirs(dst, exist_ok=True)


def vals(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if "step_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return [float(r["Counter_Value"]) for r in rows]


fetch = vals(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
write = vals(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
cfg = bench["config"]
f_kb, w_kb = statistics.median(fetch[1:] or fetch), statistics.median(write[1:] or write)
out = {
    "kernel": bench["roofline"]["kernel"], "build_id": bench["roofline"]["build_id"],
    "topology": cfg["topology"], "replicas": cfg["replicas_per_gpu"], "hops": cfg["hops_per_step"],
    "fetch_size_kb_median": f_kb, "write_size_kb_median": w_kb,
    "read_bytes_per_launch": 2 * f_kb * 1024, "write_bytes_per_launch": w_kb * 1024,
    "bytes_per_launch": 2 * f_kb * 1024 + w_kb * 1024,
    "correction": "read x2 (gfx950 FETCH_SIZE half-count for 16-B/lane streaming reads); writes as measured",
    "dispatches": len(fetch), "tag": tag,
}
path = os.path.join(root, "profiles", "pmc_traffic.json")
try:
    old = json.load(open(path))
    entries = old.get("entries", [old] if "kernel" in old else [])
except (OSError, ValueError):
    entries = []
key = lambda e: (e["topology"], e["replicas"], e["hops"])
entries = [e for e in entries if key(e) != key(out)] + [out]
json.dump({"entries": entries}, open(path, "w"), indent=1)

sq = {}
for sub in ("a", "b", "c"):
    f = os.path.join(src, "sq", sub, "run_counter_collection.csv")
    if os.path.exists(f):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                sq.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
if sq:
    med = {k: statistics.median(v[1:] or v) for k, v in sq.items()}
    hops = bench["roofline"]["hops_per_launch"]
    e = {k: out[k] for k in ("kernel", "build_id", "topology", "replicas", "hops", "tag")}
    if "GRBM_GUI_ACTIVE" in med:
        cyc = med["GRBM_GUI_ACTIVE"] / 8
        if "SQ_INSTS_SALU" in med:
            e["salu_busy"] = med["SQ_INSTS_SALU"] / (cyc * 256)
        if "SQ_INSTS_VALU" in med:
            e["valu_busy"] = 2 * med["SQ_INSTS_VALU"] / (cyc * 1024)
    for k, name in (("SQ_INSTS_SALU", "salu_per_hop"), ("SQ_INSTS_VALU", "valu_per_hop"),
                    ("SQ_INSTS_BRANCH", "branch_per_hop"), ("SQ_INSTS_VMEM_RD", "vmem_rd_per_hop"),
                    ("SQ_INSTS_LDS", "lds_per_hop"), ("SQ_LDS_BANK_CONFLICT", "lds_conflict_per_hop")):
        if k in med:
            e[name] = med[k] / hops
    if "SQ_WAVE_CYCLES" in med:
        e["wait_mem_frac"] = med.get("SQ_WAIT_ANY", 0) / med["SQ_WAVE_CYCLES"]
        e["wait_dep_frac"] = med.get("SQ_WAIT_INST_ANY", 0) / med["SQ_WAVE_CYCLES"]
    e["counters_median"] = med
    path_sq = os.path.join(root, "profiles", "pmc_sq.json")
    try:
        sq_entries = json.load(open(path_sq)).get("entries", [])
    except (OSError, ValueError):
        sq_entries = []
    sq_entries = [x for x in sq_entries if key(x) != key(e)] + [e]
    json.dump({"entries": sq_entries}, open(path_sq, "w"), indent=1)
    print(json.dumps({k: v for k, v in e.items() if k != "counters_median"}, indent=1))
shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
shutil.copy(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), os.path.join(dst, "pmc_fetch_size.csv"))
shutil.copy(os.path.join(src, "pmc_write", "run_counter_collection.csv"), os.path.join(dst, "pmc_write_size.csv"))
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
for sub in ("a", "b", "c"):                     # SQ instruction-mix / stall passes (scripts/pmc_sq.sh)
    f = os.path.join(src, "sq", sub, "run_counter_collection.csv")
    if os.path.exists(f):
        shutil.copy(f, os.path.join(dst, f"pmc_sq_{sub}.csv"))
print(json.dumps(out, indent=1))
