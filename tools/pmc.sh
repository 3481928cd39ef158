# PMC counters per kernel, one pass per counter group (rocprofv3 --pmc with
# --kernel-trace only), on a 256 MiB bench run.  Output: gpurun_out/pmc/pass*/
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $2 --output-format csv -d $R/gpurun_out/pmc/$1 -o run -- \
    python3 $R/bench.py --steps 1 --warmup 1 --mib 256 --no-cpu --no-verify > $R/gpurun_out/pmc_$1.log 2>&1
}
run p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" && \
run p2 "FETCH_SIZE" && run p3 "WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
