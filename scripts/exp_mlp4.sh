set -e
T="timeout -k 10 300"
B="timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 3 --warmup 1"
for lib in w8 w16; do
  export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_$lib.so
  $T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_mem_engine.py -k "mlp or dqn or buffer" > gpurun_out/e6_${lib}_tests.log 2>&1
  $B --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --hops 1024 > gpurun_out/e6_${lib}_c4.json
  $B --topology abilene_on_geant --policy dqn_buffer --hops 1024 > gpurun_out/e6_${lib}_c3.json
  $B --topology er256 --policy dqn_buffer --warmup 13 > gpurun_out/e6_${lib}_c5.json
done
