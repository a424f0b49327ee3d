# A/B: prisma_amd/_ablate/libprisma_amd_base.so (previous build) vs the working tree's library,
# alternating on one box.  Usage: bash scripts/ab_lib.sh <bench args...>
ARGS="$*"
for i in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_base.so; else unset PRISMA_LIB; fi
    timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 5 --warmup 1 $ARGS | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']/1e6,1), round(d['roofline']['kernel_ms'],2))" || exit 1
  done
done
