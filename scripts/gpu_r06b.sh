#!/bin/bash
# Round 6 analysis counters on the build in tree: SQ instruction mix of the headline and config 3,
# and config 5's L2 hit / miss / fabric-request split for the DQN-buffer policy against the SP table.
OUT=gpurun_out/r06b
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
K="--kernel-include-regex step_kernel -f csv"
SQA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH"
TCC="TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_EA0_RDREQ_sum"
TCC2="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
run() { echo "== $1"; timeout -s KILL 240 rocprofv3 --pmc $2 $K -d $OUT/$1 -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 $3 > $OUT/$1.log 2>&1; rc=$?; tail -c 400 $OUT/$1.log | tail -2; return $rc; }
run hl_sqa "$SQA" "--preset config2" && \
run aog_sqa "$SQA" "--preset config3" && \
run er_dqn_tcc "$TCC" "--preset config5 --warmup 4" && \
run er_sp_tcc "$TCC" "--preset config5 --policy sp --warmup 4" && \
run er_dqn_tcc2 "$TCC2" "--preset config5 --warmup 4" && \
run er_sp_tcc2 "$TCC2" "--preset config5 --policy sp --warmup 4"
echo rc=$?
