mkdir -p gpurun_out/scal
for R in 1024 2048 3072 4096 8192; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 --replicas $R > gpurun_out/scal/r$R.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/scal/r$R.json')); print($R, round(d['value']/1e6,1), 'Mhops/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done
