set -e
T="timeout -k 10 600"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mem_engine.py tests/test_gpu_parity.py -k "mem or er256 or weights_change" > gpurun_out/e20_tests.log 2>&1
B="timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 5 --warmup 13"
$B --topology er256 --policy dqn_buffer > gpurun_out/e20_c5.json
$B --topology er256 --policy sp > gpurun_out/e20_c5sp.json
