#!/bin/bash
# One bench line per BASELINE.json config that fits one GPU, appended to
# gpurun_out/configs.jsonl.  Config 4 runs its per-GPU share (16384 / 8 = 2048 replicas)
# across the load-factor sweep; config 5 (ER-256, memory-resident engine) its per-GPU share
# (8192 / 8 = 1024 replicas).
set -e
OUT=gpurun_out/configs.jsonl
: > $OUT
B="timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 5 --warmup 1"
echo "config 1: abilene SP, 1 replica" && $B --policy sp --replicas 1 --hops 2048 >> $OUT
echo "config 2: abilene DQ-routing, 4096" && $B >> $OUT
echo "config 3: abilene on geant, DQN-buffer pingAsObs=1, 4096" && $B --topology abilene_on_geant --policy dqn_buffer >> $OUT
echo "config 3 (SP table)" && $B --topology abilene_on_geant --policy sp >> $OUT
for lf in 0.5 0.75 1.0 1.25 1.5 1.75 2.0; do
  echo "config 4: geant DQN-buffer pingAsObs=0 lf $lf, 2048" && $B --topology geant --policy dqn_buffer --ping-as-obs 0 --load-factor $lf --replicas 2048 >> $OUT
done
echo "config 4 variant: geant DQN-buffer pingAsObs=1 lf 1.0, 2048" && $B --topology geant --policy dqn_buffer --ping-as-obs 1 --replicas 2048 >> $OUT
# ER-256: bench.py's defaults (1 024 replicas, 8 192 hops/step, 13 warmup steps past the
# first simulated second's flow-start transient)
echo "config 5: ER-256 DQN-buffer pingAsObs=1, 1024" && $B --topology er256 --policy dqn_buffer --warmup 13 >> $OUT
echo "config 5 (SP table)" && $B --topology er256 --policy sp --warmup 13 >> $OUT
python - <<'PY'
import json
for l in open("gpurun_out/configs.jsonl"):
    d = json.loads(l)
    print(f"{d['config']['workload'][:110]:110s} {d['value']:.3e} hops/s  kernel {d['roofline']['kernel_ms']:.2f} ms  err {d['errors']}")
PY
