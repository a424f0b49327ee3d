#!/bin/bash
# tunnel parity tests first (all reported), then the full GPU suite and the headline bench;
# anything but a clean pass / plain test failure (exit 0 / 1) ends the script.
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -k tunnel --timeout=300 > gpurun_out/tests_tunnel.log 2>&1
rc=$?
tail -30 gpurun_out/tests_tunnel.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout=300 -k "not tunnel" > gpurun_out/tests_all.log 2>&1
rc2=$?
tail -5 gpurun_out/tests_all.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err
rc3=$?
cat gpurun_out/bench_t.json | head -c 600
exit $((rc + rc2 + rc3))
