#!/bin/bash
# Build a diagnostic variant of the engine library with extra compiler flags into
# prisma_amd/_ablate/libprisma_amd_<name>.so (all translation units, the product's flags).
# Usage: bash scripts/build_variant.sh <name> [-DFLAG ...]; then on the GPU box
# bash scripts/ab_libs.sh "<name> ..." <bench args>.  Results of -DPRISMA_ABLATE builds are
# not parity results.  SRC_DIR=<dir> compiles the sources of another tree (e.g. a git archive of HEAD).
set -e
NAME=$1; shift
O=/tmp/prisma_variant_$NAME
rm -rf $O                                    # never link a stale object of an earlier run
mkdir -p $O prisma_amd/_ablate
FLAGS=$(python -c "from prisma_amd import buildid; print(' '.join(buildid.HIPCC_FLAGS))")
SRCS=$(python -c "from prisma_amd import buildid; print(' '.join(buildid.ENGINE_SOURCES))")
PIDS=()
for f in $SRCS; do
  # ONLY=<source>: that translation unit alone, the others from the in-tree objects of the last
  # build_engine (same sources; quick memory-engine experiments)
  # (ONLY may list several translation units, space-separated)
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $f "* ]]; then cp prisma_amd/csrc/${f%.hip}.o $O/; continue; fi
  /opt/rocm/bin/hipcc $FLAGS -DPRISMA_BUILD_ID="\"variant-$NAME\"" "$@" -c -o $O/${f%.hip}.o ${SRC_DIR:-prisma_amd/csrc}/$f &
  PIDS+=($!)
done
for p in "${PIDS[@]}"; do
  wait $p || { echo "hipcc failed (variant $NAME)" >&2; exit 1; }
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o prisma_amd/_ablate/libprisma_amd_$NAME.so $O/*.o
echo built prisma_amd/_ablate/libprisma_amd_$NAME.so
