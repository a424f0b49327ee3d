set -e
T="timeout -k 10 600"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_mem_engine.py tests/test_trainer.py > gpurun_out/e15_tests.log 2>&1
B="timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 5 --warmup 1"
$B --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --hops 1024 > gpurun_out/e15_c4.json
$B --topology abilene_on_geant --policy dqn_buffer --hops 1024 > gpurun_out/e15_c3.json
$B --topology er256 --policy dqn_buffer --warmup 13 > gpurun_out/e15_c5.json
