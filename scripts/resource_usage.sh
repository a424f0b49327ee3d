#!/bin/bash
# Per-kernel register / spill / LDS / occupancy report of the engine's step kernels
# (device-only compile with the product's flags + -Rpass-analysis=kernel-resource-usage).
# Usage: bash scripts/resource_usage.sh [source ...] [-- extra hipcc flags]; default: all sources.
cd "$(dirname "$0")/.."
SRCS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SRCS+=("$1"); shift; done
[ "$1" == "--" ] && shift
[ ${#SRCS[@]} -eq 0 ] && SRCS=(prisma_engine_lite.hip prisma_engine.hip prisma_engine_mem.hip)
FLAGS=$(python -c "from prisma_amd import buildid; print(' '.join(buildid.HIPCC_FLAGS))")
for f in "${SRCS[@]}"; do
  /opt/rocm/bin/hipcc $FLAGS "$@" --cuda-device-only -c -o /dev/null -Rpass-analysis=kernel-resource-usage \
      prisma_amd/csrc/$f 2>&1 | python scripts/resource_summary.py
done
