"""Host timeline of the unit protocol (bz2mi.shard.compress_units trace):
per-hop latency of the chain token, the chain's share of the critical path,
the seed rounds, and a model of the N-GPU critical path.

  python tools/unit_hops.py <prefix>            # traces <prefix>.<rank>.json (bench.py, BZ2MI_UNIT_TRACE)
  python tools/unit_hops.py --cpu-world 8 out   # gloo CPU ranks on cpu_ref units, then the analysis

A hop is the time from unit g-1's chain end (on its rank) to unit g's token
arrival (on the next rank): gloo send + the receiver's wait.  All ranks run
on one host, so perf_counter (CLOCK_MONOTONIC) is one clock.
"""
from __future__ import annotations

import glob
import json
import os
import socket
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def analyse(prefix: str) -> dict:
    runs = [json.load(open(f)) for f in sorted(glob.glob(prefix + ".*.json"))]
    assert runs, prefix
    owners = runs[0]["owners"]
    ev = {}
    t0 = min(e[2] for r in runs for e in r["events"] if e[0] == "step")
    for r in runs:
        for name, g, t in r["events"]:
            ev.setdefault(name, {})[(g, r["rank"]) if name in ("round", "step", "end") else g] = t - t0
    chain, recv = ev.get("chain", {}), ev.get("recv", {})
    hops = [recv[g] - chain[g - 1] for g in range(1, len(owners)) if g in recv and g - 1 in chain]
    # a chain's own time: from its token (or the previous local chain) to its end
    own = []
    for g in range(len(owners)):
        if g not in chain:
            continue
        start = recv.get(g, chain.get(g - 1, 0.0))
        own.append(chain[g] - start)
    ends = [t for (g, r), t in ev.get("end", {}).items()]
    out = {
        "world": runs[0]["world"], "units": len(owners), "unit_bytes": runs[0]["unit_bytes"],
        "hop_ms": {"n": len(hops), "median": round(statistics.median(hops) * 1e3, 3) if hops else None,
                   "max": round(max(hops) * 1e3, 3) if hops else None},
        "chain_ms": {"median": round(statistics.median(own) * 1e3, 3) if own else None},
        "last_chain_end_ms": round(max(chain.values()) * 1e3, 3) if chain else None,
        "step_ms": round(max(ends) * 1e3, 3) if ends else None,
        "rounds_ms": sorted(round(t * 1e3, 3) for (j, r), t in ev.get("round", {}).items() if r == 0),
    }
    if hops and own:
        n = len(owners)
        out["model_chain_path_ms"] = round((n - 1) * (statistics.median(hops) + statistics.median(own)) * 1e3, 3)
    return out


def _cpu_rank(rank, world, port, prefix, nunits):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    sys.path.insert(0, os.path.join(REPO, "bzip2-opencl_amd"))
    import time

    import torch.distributed as dist
    from conftest import CpuRefUnit, unit_buffers

    import bz2mi
    from bz2mi import shard, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    U = 1 << 20
    data = synth.random_bytes(U * nunits).tobytes()
    cuts = [U * k for k in range(1, nunits)]
    bufs = unit_buffers(data, cuts, bz2mi.unit_halo(9, 10000))
    owners = shard.interleaved_owners(len(bufs), world)
    units = {}
    for g, (buf, n_own, n_halo, ends) in enumerate(bufs):
        if owners[g] == rank:
            u = CpuRefUnit(9, 10, 10000, threads=1)
            u.begin(buf, n_own, n_halo, ends)
            units[g] = u
    dist.barrier()
    trace = [("step", -1, time.perf_counter())]
    shard.compress_units(units, owners, 10, 9, group=None, speculate="never", trace=trace)
    trace.append(("end", -1, time.perf_counter()))
    with open(f"{prefix}.{rank}.json", "w") as f:
        json.dump({"rank": rank, "world": world, "units": len(bufs), "unit_bytes": U, "owners": owners,
                   "events": trace}, f)
    dist.barrier()
    dist.destroy_process_group()


def main():
    args = sys.argv[1:]
    if args and args[0] == "--cpu-world":
        import torch.multiprocessing as mp
        world, prefix = int(args[1]), args[2]
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_cpu_rank, args=(r, world, port, prefix, 4 * world)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join()
        assert all(p.exitcode == 0 for p in procs)
    else:
        prefix = args[0]
    print(json.dumps(analyse(prefix), indent=1))


if __name__ == "__main__":
    main()
