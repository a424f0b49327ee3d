set -e
T="timeout -k 10 600"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mem_engine.py > gpurun_out/e11_tests.log 2>&1
B="timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 3 --warmup 13"
$B --topology er256 --policy dqn_buffer > gpurun_out/e11_c5.json
