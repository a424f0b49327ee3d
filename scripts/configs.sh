#!/bin/bash
# One bench line per BASELINE.json config that fits one GPU, appended to
# gpurun_out/configs.jsonl, through bench.py's presets (per-GPU shares: config 4's 16384 / 8 = 2048
# GEANT replicas over its load-factor sweep, config 5's 8192 / 8 = 1024 ER-256 replicas).
# CPU=1: each line also carries its cpu_baseline (the oracle on this host's threads, same workload).
set -e
OUT=gpurun_out/configs.jsonl
: > $OUT
C=${CPU:-0}
B="timeout -k 10 600 python bench.py --steps 5 --warmup 1"
echo "config 1: abilene SP, 1 replica" && $B --preset config1 --cpu-baseline $C >> $OUT
echo "config 2: abilene DQ-routing, 4096" && $B --preset config2 --cpu-baseline $C >> $OUT
echo "config 3: abilene on geant, DQN-buffer pingAsObs=1, 4096" && $B --preset config3 --cpu-baseline $C >> $OUT
echo "config 3 (SP table)" && $B --preset config3 --policy sp --cpu-baseline 0 >> $OUT
echo "config 4: geant DQN-buffer pingAsObs=0, 2048, lf 0.5 ... 2.0" && $B --preset config4 --cpu-baseline $C >> $OUT
echo "config 4 variant: geant DQN-buffer pingAsObs=1 lf 1.0, 2048" && $B --preset config4 --ping-as-obs 1 --load-factors 1.0 --cpu-baseline 0 >> $OUT
# ER-256: the preset's 4 warmup steps (32 768 hops each) pass the first simulated second's flow-start transient
echo "config 5: ER-256 DQN-buffer pingAsObs=1, 1024" && $B --preset config5 --warmup 4 --cpu-baseline $C >> $OUT
echo "config 5 (SP table)" && $B --preset config5 --policy sp --warmup 4 --cpu-baseline 0 >> $OUT
python - <<'PY'
import json
for l in open("gpurun_out/configs.jsonl"):
    d = json.loads(l)
    cb = d.get("cpu_baseline")
    cpu = f"  cpu {cb['value']:.3e} ({cb['cores']} thr, 1-thr {cb['value_1core']:.3e})" if cb else ""
    print(f"{d['config']['workload'][:100]:100s} {d['value']:.3e} hops/s  kernel {d['roofline']['kernel_ms']:.2f} ms  err {d['errors']}{cpu}")
PY
