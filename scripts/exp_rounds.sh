# occupancy rounds: LDS allows 7 replicas per CU for GEANT+MLP and Abilene-on-GEANT
set -e
B="timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 3 --warmup 1"
for R in 1792 2048; do $B --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas $R --hops 1024 > gpurun_out/e9_c4_$R.json; done
for R in 3584 4096; do $B --topology abilene_on_geant --policy sp --replicas $R > gpurun_out/e9_c3_$R.json; done
