#!/bin/bash
# Instruction- and scalar-cache counters plus average in-flight levels of the step kernel, one
# rocprofv3 --pmc pass each (no trace domains), for one bench configuration.
# Usage (on the GPU box): bash scripts/pmc_cache.sh <tag> [bench args]
TAG=${1:-x}
shift || true
OUT=gpurun_out/pmc_cache_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="python bench.py --steps 5 --cpu-baseline 0 $*"
K="--kernel-include-regex step_kernel -f csv"
timeout -s KILL 180 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES $K -d $OUT/a -o run -- $B > $OUT/a.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS $K -d $OUT/b -o run -- $B > $OUT/b.log 2>&1 || exit $?
python - "$OUT" <<'PY'
import csv, glob, statistics, sys, collections
out = sys.argv[1]
v = collections.defaultdict(list)
for f in glob.glob(out + "/*/run_counter_collection.csv") + glob.glob(out + "/*/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        v[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: statistics.median(x) for k, x in v.items()}
for k in sorted(m): print(f"{k:24s} {m[k]:.4g}")
def ratio(a, b): return m[a] / m[b] if m.get(b) else float("nan")
print("icache miss rate", ratio("SQC_ICACHE_MISSES", "SQC_ICACHE_HITS"))
print("dcache miss rate", ratio("SQC_DCACHE_MISSES", "SQC_DCACHE_HITS"))
print("smem latency (cycles, level/insts)", ratio("SQ_INST_LEVEL_SMEM", "SQ_INSTS_SMEM"))
print("vmem-read latency (cycles, level/insts)", ratio("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM_RD"))
print("ifetch latency (cycles, level/fetches)", ratio("SQ_IFETCH_LEVEL", "SQ_IFETCH"))
PY
