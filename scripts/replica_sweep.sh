# Replicas per GPU vs throughput: the headline (Abilene, 16 replicas per CU fit at once) and
# config 4 (GEANT + DQN-buffer, 8 per CU: 2 048 fill the chip once, more run in rounds)
mkdir -p gpurun_out/scal
for R in 1024 2048 3072 4096 6144 8192; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 5 --warmup 1 --replicas $R > gpurun_out/scal/r$R.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/scal/r$R.json')); print('abilene', $R, round(d['value']/1e6,1), 'Mhops/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done
for R in 1024 1792 2048 2304 3584 4096; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 3 --warmup 1 --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas $R > gpurun_out/scal/g$R.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/scal/g$R.json')); print('geant-mlp', $R, round(d['value']/1e6,1), 'Mhops/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done
