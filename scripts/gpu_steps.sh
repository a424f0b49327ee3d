#!/bin/bash
# Run GPU steps in order; a step that ends in a fault, abort, segfault, time limit or hang
# (any exit status other than 0 = pass or 1 = failed assertions) ends the call there.
# Usage: bash scripts/gpu_steps.sh "<step 1>" "<step 2>" ...
mkdir -p gpurun_out
for s in "$@"; do
  echo "== $s"
  bash -c "$s"
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "== step ended with status $rc: stopping"; exit $rc; fi
done
