#!/bin/bash
# Unit-protocol host timelines on one MI355X: 8 ranks sharing cuda:0 over gloo
# (BZ2MI_SHARE_GPU=1), 4 units each, seed sums by all-gather rounds and by the
# token; tools/unit_hops.py turns the traces into per-hop latency and the
# modelled critical path.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r6hops}
mkdir -p $O
MIB=${MIB:-128}
for seeds in rounds token; do
  BZ2MI_SHARE_GPU=1 BZ2MI_SEEDS=$seeds BZ2MI_UNIT_TRACE=$O/tr_$seeds timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) $R/bench.py --gpus 8 --mib $MIB --units-per-gpu 4 --steps 3 --warmup 1 --no-cpu --no-verify > $O/bench_$seeds.json 2> $O/bench_$seeds.err || { echo FAILED $seeds; tail -20 $O/bench_$seeds.err; exit 1; }
  python3 $R/tools/unit_hops.py $O/tr_$seeds > $O/hops_$seeds.json || exit 1
  echo "$seeds: $(cat $O/hops_$seeds.json | tr -d '\n ')"
done
