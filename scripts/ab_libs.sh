# A/B of several prebuilt libraries (prisma_amd/_ablate/libprisma_amd_<name>.so), alternating
# on one box.  Usage: bash scripts/ab_libs.sh "<names>" <bench args...>
NAMES="$1"; shift
ARGS="$*"
for i in 1 2; do
  for lib in $NAMES; do
    export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_$lib.so
    timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 5 --warmup 1 $ARGS | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']/1e6,1), round(d['roofline']['kernel_ms'],2))" || exit 1
  done
done
