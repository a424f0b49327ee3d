#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the step kernel for several libraries (prisma_amd/_ablate/libprisma_amd_<name>.so;
# "new" = the in-tree library) on one workload: traffic attribution by ablation (-DPRISMA_ABLATE builds
# are diagnostics, not parity results).  Usage: bash scripts/traffic_ab.sh <tag> "<libs>" <bench args...>
TAG=$1; LIBS=$2; shift 2
OUT=gpurun_out/traffic_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="python bench.py --steps 3 --warmup 1 --cpu-baseline 0 $*"
for lib in $LIBS; do
  if [ $lib = new ]; then unset PRISMA_LIB; else export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_$lib.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex step_kernel -f csv -d $OUT/${lib}_$c -o run -- $B > $OUT/${lib}_$c.log 2>&1 || exit 1
  done
  python - $OUT $lib <<'PY'
import csv, statistics, sys
out, lib = sys.argv[1], sys.argv[2]
v = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = [float(r["Counter_Value"]) for r in csv.DictReader(open(f"{out}/{lib}_{c}/run_counter_collection.csv"))
            if "step_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c]
    v[c] = statistics.median(rows[1:] or rows)
print(f"{lib:10s} read {2 * v['FETCH_SIZE'] * 1024 / 1e9:7.3f} GB  write {v['WRITE_SIZE'] * 1024 / 1e9:7.3f} GB per launch")
PY
done
