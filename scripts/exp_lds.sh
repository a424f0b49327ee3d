set -e
T="timeout -k 10 600"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_mem_engine.py tests/test_ns3env.py > gpurun_out/e10_tests.log 2>&1
B="timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 3 --warmup 1"
$B --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --hops 1024 > gpurun_out/e10_c4.json
$B --topology abilene_on_geant --policy dqn_buffer --hops 1024 > gpurun_out/e10_c3.json
$B --topology abilene_on_geant --policy sp > gpurun_out/e10_c3sp.json
$B > gpurun_out/e10_c2.json
