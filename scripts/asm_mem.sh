#!/bin/bash
# Assembly of the memory-resident DQN-buffer step kernel (prisma_mem_step_kernel<true, false>, config 5)
# with register counts and instruction-class counts.  Usage: bash scripts/asm_mem.sh [out.s] [-D...]
cd "$(dirname "$0")/.."
OUT=${1:-/tmp/mem.s}; shift
FLAGS=$(python -c "from prisma_amd import buildid; print(' '.join(buildid.HIPCC_FLAGS))")
/opt/rocm/bin/hipcc $FLAGS "$@" --cuda-device-only -S -o $OUT prisma_amd/csrc/prisma_engine_mem.hip 2>/dev/null || exit 1
python - "$OUT" <<'PY'
import re, sys, collections
txt = open(sys.argv[1]).read()
name = "_Z22prisma_mem_step_kernelILb1ELb0EEv7KParams"
m = re.search(rf"^{name}:.*?\n(.*?)^\s*s_endpgm", txt, re.S | re.M)
ins = [l.strip().split()[0] for l in m.group(1).splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
c = collections.Counter(ins)
print(f"instructions {len(ins)}  s_nop {c['s_nop']}  v_accvgpr_read {c['v_accvgpr_read_b32']}  v_accvgpr_write {c['v_accvgpr_write_b32']}  "
      f"v_readlane {c['v_readlane_b32']}  v_writelane {c['v_writelane_b32']}  v_mov {c['v_mov_b32_e32']}  global_load {sum(v for k, v in c.items() if k.startswith('global_load'))}")
blocks = re.split(r"\n\s+- \.agpr_count:", txt)
md = next(("agpr_count:" + b_) for b_ in blocks if re.search(rf"\.name:\s+{name}\s", b_))
for k in ("agpr_count", "vgpr_count", "sgpr_count", "sgpr_spill_count", "vgpr_spill_count"):
    mm = re.findall(rf"{k}:\s+(\d+)", md)
    print(k, mm[0] if mm else None)
PY
