set -e
T="timeout -k 10 200"
$T python scripts/timing.py run --topology abilene_on_geant --policy sp --replicas 4096 --hops 1024 > gpurun_out/e18_t_aog_sp.txt
$T python scripts/timing.py run --topology abilene --policy dq_routing --replicas 4096 --hops 2048 > gpurun_out/e18_t_ab.txt
$T python scripts/timing.py run --topology geant --policy dq_routing --ping-as-obs 0 --replicas 2048 --hops 1024 > gpurun_out/e18_t_geant_tab.txt
