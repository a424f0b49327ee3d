set -e
T="timeout -k 10 200"
B="$T python bench.py --cpu-baseline 0 --steps 3 --warmup 1"
$B --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --hops 1024 > gpurun_out/e1_geant_mlp.json
$B --topology geant --policy dq_routing --ping-as-obs 0 --replicas 2048 --hops 1024 > gpurun_out/e1_geant_tab.json
$B --policy dqn_buffer --hops 1024 > gpurun_out/e1_ab_mlp.json
$T python scripts/timing.py run --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --hops 512 > gpurun_out/e1_t_geant_mlp.txt
$T python scripts/timing.py run --topology geant --policy dq_routing --ping-as-obs 0 --replicas 2048 --hops 512 > gpurun_out/e1_t_geant_tab.txt
$T python scripts/timing.py run --topology abilene --policy dqn_buffer --replicas 4096 --hops 512 > gpurun_out/e1_t_ab_mlp.txt
