set -e
T="timeout -k 10 200"
$T python scripts/timing.py run --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --hops 512 > gpurun_out/e2_t_geant_mlp.txt
$T python scripts/timing.py run --topology abilene --policy dqn_buffer --replicas 4096 --hops 512 > gpurun_out/e2_t_ab_mlp.txt
$T python scripts/timing.py run --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 256 --hops 512 > gpurun_out/e2_t_geant_mlp256.txt
