#!/bin/bash
# PMC passes (SQ instruction mix / waits, LDS, L2) for one workload (DATA), 256 MiB
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=${DATA:-text}
O=$R/gpurun_out/pmc_${TAG:-r2}_$D
mkdir -p $O
run() {
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $2 --output-format csv -d $O/$1 -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --mib 256 --data $D --no-cpu --no-verify > $O/$1.log 2>&1 || { echo "PASS $1 FAILED"; tail -5 $O/$1.log; exit 1; }
}
run p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU TCC_HIT_sum TCC_MISS_sum"
run p3 "SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
echo done
