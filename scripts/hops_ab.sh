export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_r04a.so
for i in 1 2; do
  for h in 8192 16384; do
    s=$(( 20 * 8192 / h )); w=$(( 5 * 8192 / h ))
    timeout -k 10 200 python bench.py --cpu-baseline 0 --hops $h --steps $s --warmup $w | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('hops $h', round(d['value']/1e6,1), 'Mhops/s kernel', round(d['roofline']['kernel_ms'],2), 'step', round(d['ms_per_step'],2))" || exit 1
  done
done
