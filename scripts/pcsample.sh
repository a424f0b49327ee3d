#!/bin/bash
# Instruction-level hot spots of the step kernel: rocprofv3's PC sampling (host-trap method,
# time interval) over a short bench run, then scripts/pcsample_report.py maps the sampled
# program counters to the kernel's disassembly.  The supported configurations are listed first
# (rocprofv3 -L); the sampling run is skipped when host-trap sampling is not offered.
# Usage (on the GPU box): bash scripts/pcsample.sh <tag> [extra bench args]
TAG=${1:-x}
shift || true
OUT=gpurun_out/pcs_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 -L > $OUT/list.txt 2>&1
grep -i -n "pc.sampl\|host_trap\|stochastic" $OUT/list.txt | head -20
if ! grep -qi "host_trap" $OUT/list.txt; then echo "no host-trap PC sampling on this box"; exit 0; fi
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
  --pc-sampling-unit time --pc-sampling-interval 1000 -f csv -d $OUT/run -o run -- \
  python bench.py --steps 3 --warmup 1 --cpu-baseline 0 "$@" > $OUT/run.log 2>&1
rc=$?
tail -5 $OUT/run.log
find $OUT -name "*.csv" | head
exit $rc
