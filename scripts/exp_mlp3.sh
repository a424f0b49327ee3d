set -e
T="timeout -k 10 300"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_mem_engine.py -k "mlp or dqn or buffer" > gpurun_out/e5_tests.log 2>&1
B="timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 3 --warmup 1"
$B --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --hops 1024 > gpurun_out/e5_c4.json
$B --topology abilene_on_geant --policy dqn_buffer --hops 1024 > gpurun_out/e5_c3.json
$B --policy dqn_buffer --hops 1024 > gpurun_out/e5_ab.json
$B --topology er256 --policy dqn_buffer --warmup 13 > gpurun_out/e5_c5.json
T="timeout -k 10 200"
$T python scripts/timing.py run --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --hops 512 > gpurun_out/e5_t_geant_mlp.txt
$T python scripts/timing.py run --topology er256 --policy dqn_buffer --replicas 1024 --hops 8192 --warm 13 > gpurun_out/e5_t_er_mlp.txt
