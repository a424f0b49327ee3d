#!/bin/bash
# (_ab_old/ is listed in .gpurunignore to keep pushes small: remove that line before using this script; scripts/ab_lib.sh compares prebuilt libraries instead)
# A/B throughput: _ab_old/ (a previous tree, built) vs the working tree, alternating, same box.
ARGS="$*"
for i in 1 2; do
  (cd _ab_old && timeout -k 10 200 python bench.py --cpu-baseline 0 $ARGS | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('old', round(d['value']/1e6,1), round(d['roofline']['kernel_ms'],2))") || exit 1
  timeout -k 10 200 python bench.py --cpu-baseline 0 $ARGS | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('new', round(d['value']/1e6,1), round(d['roofline']['kernel_ms'],2))" || exit 1
done
