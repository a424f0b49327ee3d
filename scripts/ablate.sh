#!/bin/bash
# Diagnostic timing of engine parts: builds -DPRISMA_ABLATE=<mask> variants
# (results are NOT parity results) and runs one bench line per variant.
# Usage: on this container `bash scripts/ablate.sh build`, on the GPU box `bash scripts/ablate.sh run [bench args]`.
set -e
D=gpurun_out/ablate
SRC=prisma_amd/csrc/prisma_engine.hip
if [ "$1" = build ]; then
  mkdir -p prisma_amd/_ablate
  for m in 1 2 4 7; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -std=c++17 -DPRISMA_ABLATE=$m \
      -o prisma_amd/_ablate/libprisma_amd_a$m.so $SRC &
  done
  wait
  exit 0
fi
shift
mkdir -p $D
timeout -k 10 200 python bench.py --cpu-baseline 0 "$@" > $D/base.json 2> $D/base.err
for m in 1 2 4 7; do
  PRISMA_LIB=prisma_amd/_ablate/libprisma_amd_a$m.so timeout -k 10 200 python bench.py --cpu-baseline 0 "$@" > $D/a$m.json 2> $D/a$m.err
done
for f in base a1 a2 a4 a7; do python -c "import json,sys; d=json.load(open('$D/$f.json')); print('$f', round(d['value']/1e6,1), 'Mhops/s', round(d['roofline']['kernel_ms'],2), 'ms')"; done
