# L2 hit rate and L1->L2 read latency of the step kernel (config 4 DQN-buffer vs table)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for pol in dqn_buffer dq_routing; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --kernel-include-regex step_kernel -f csv -d gpurun_out/l2_$pol -o run -- python bench.py --cpu-baseline 0 --steps 2 --warmup 1 --topology geant --policy $pol --ping-as-obs 0 --replicas 2048 --hops 512 > gpurun_out/l2_$pol.log 2>&1
done
python - <<'PY'
import csv, collections
for pol in ("dqn_buffer", "dq_routing"):
    t = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/l2_{pol}/run_counter_collection.csv")):
        t[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sorted(v)[len(v)//2] for k, v in t.items()}
    print(pol, {k: f"{v:.3e}" for k, v in m.items()},
          "hit", m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]),
          "lat", m["TCP_TCC_READ_REQ_LATENCY_sum"] / m["TCP_TCC_READ_REQ_sum"])
PY
