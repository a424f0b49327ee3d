set -e
B="timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 5 --warmup 1"
for h in 2048 4096 8192; do $B --hops $h > gpurun_out/e16_h$h.json; done
