#!/bin/bash
# Build a diagnostic variant of the engine library with extra compiler flags into
# prisma_amd/_ablate/libprisma_amd_<name>.so (all translation units, the product's flags).
# Usage: bash scripts/build_variant.sh <name> [-DFLAG ...]; then on the GPU box
# bash scripts/ab_libs.sh "<name> ..." <bench args>.  Results of -DPRISMA_ABLATE builds are
# not parity results.
set -e
NAME=$1; shift
O=/tmp/prisma_variant_$NAME
mkdir -p $O prisma_amd/_ablate
FLAGS=$(python -c "from prisma_amd import buildid; print(' '.join(buildid.HIPCC_FLAGS))")
SRCS=$(python -c "from prisma_amd import buildid; print(' '.join(buildid.ENGINE_SOURCES))")
for f in $SRCS; do
  /opt/rocm/bin/hipcc $FLAGS -DPRISMA_BUILD_ID="\"variant-$NAME\"" "$@" -c -o $O/${f%.hip}.o prisma_amd/csrc/$f &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o prisma_amd/_ablate/libprisma_amd_$NAME.so $O/*.o
echo built prisma_amd/_ablate/libprisma_amd_$NAME.so
