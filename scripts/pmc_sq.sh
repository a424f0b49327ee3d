#!/bin/bash
# SQ instruction-mix and stall counters for prisma_step_kernel (separate passes).
OUT=gpurun_out/sq_${1:-x}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="python bench.py --steps 3 --warmup 1 --cpu-baseline 0"
timeout -k 10 300 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --kernel-include-regex prisma_step -f csv -d $OUT/a -o run -- $B > $OUT/a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex prisma_step -f csv -d $OUT/b -o run -- $B > $OUT/b.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex prisma_step -f csv -d $OUT/c -o run -- $B > $OUT/c.log 2>&1
echo rc=$?
tail -3 $OUT/*.log
