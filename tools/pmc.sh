# PMC counters per kernel, one pass per counter group (rocprofv3 --pmc with
# --kernel-trace only), on a 256 MiB bench run (DATA=random|text|mixed,
# EXTRA= more bench args).  Output: gpurun_out/pmc_<data>/pass*/
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=${DATA:-random}
run() {
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $2 --output-format csv -d $R/gpurun_out/pmc_$D/$1 -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --mib 256 --data $D --no-cpu --no-verify --no-900k $EXTRA > $R/gpurun_out/pmc_${D}_$1.log 2>&1
}
run p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" && \
run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" && \
run p3 "FETCH_SIZE" && run p4 "WRITE_SIZE"
