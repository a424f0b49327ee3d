#!/bin/bash
# Assembly of the headline step kernel alone (-DPRISMA_DEV_HEADLINE), with instruction-class
# counts: a quick static check of what a change does to the hot kernel (spills show up as
# scratch_* and v_writelane/v_readlane pairs).  Usage: bash scripts/asm_headline.sh [out.s] [-D...]
cd "$(dirname "$0")/.."
OUT=${1:-/tmp/headline.s}; shift
FLAGS=$(python -c "from prisma_amd import buildid; print(' '.join(buildid.HIPCC_FLAGS))")
/opt/rocm/bin/hipcc $FLAGS -DPRISMA_DEV_HEADLINE "$@" --cuda-device-only -S -o $OUT prisma_amd/csrc/prisma_engine_lite.hip || exit 1
python - "$OUT" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
m = re.search(r"^_Z20prisma_step_kernel_tILi2ELi1ELb0ELb0ELb0EEv7KParams:\n(.*?)^\s*s_endpgm", txt, re.S | re.M)
body = m.group(1) if m else txt
ins = [l.strip().split()[0] for l in body.splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
cnt = lambda p: sum(1 for i in ins if i.startswith(p))
print(f"instructions {len(ins)}  scratch {cnt('scratch_')}  v_writelane {cnt('v_writelane')}  "
      f"v_readlane {cnt('v_readlane')}  s_swappc/call {cnt('s_swappc')+cnt('s_call')}  "
      f"s_ {cnt('s_')}  v_ {cnt('v_')}  ds_ {cnt('ds_')}  global_ {cnt('global_')}  s_cbranch {cnt('s_cbranch')}")
for k in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
    mm = re.findall(rf"\.{k}:\s+(\d+)", txt)
    print(k, mm[:4])
PY
