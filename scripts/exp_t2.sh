set -e
T="timeout -k 10 200"
$T python scripts/timing.py run --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --hops 512 > gpurun_out/e12_t_geant_mlp.txt
$T python scripts/timing.py run --topology er256 --policy dqn_buffer --replicas 1024 --hops 8192 --warm 13 > gpurun_out/e12_t_er_mlp.txt
$T python scripts/timing.py run --topology er256 --policy dq_routing --replicas 1024 --hops 8192 --warm 13 > gpurun_out/e12_t_er_tab.txt
