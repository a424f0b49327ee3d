set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/e24_tests.log 2>&1
echo headline; bash scripts/ab_lib.sh
echo c4; bash scripts/ab_lib.sh --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048
