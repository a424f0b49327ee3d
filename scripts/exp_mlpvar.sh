# diagnostic MLP variants (not parity-valid): 4 partial accumulators, f32 ELU
set -e
B="timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 5 --warmup 1"
for lib in default acc4 elu both; do
  if [ $lib = default ]; then unset PRISMA_LIB; else export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_$lib.so; fi
  $B --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --hops 1024 > gpurun_out/e14_${lib}_c4.json
  $B --topology er256 --policy dqn_buffer --warmup 13 > gpurun_out/e14_${lib}_c5.json
done
