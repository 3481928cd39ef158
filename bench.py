#!/usr/bin/env python3
"""bench.py -- compress throughput of the MI355X bzip2 path (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 1 GiB of random
bytes resident in HBM, compressed at -9 with the reference's block size
(S = 9 x 10,000 = 90,000 bytes, Config.hpp:30) and parallel count p = 10, to a
complete .bz2 stream in HBM.  One step = one whole stream: device RLE1 front
end + block split + CRCs, BWT, MTF/RLE2, seed carry-over, Huffman + packing,
stream assembly.  Multi-GPU (torchrun, one process per GPU): every rank
compresses its own 1 GiB object (independent .bz2 streams, no data-path
collective) -> weak scaling; timing is the max over ranks.

Prints ONE JSON line (rank 0) with the contract fields plus `roofline` (the
dominant kernel against the HBM roofline) and `cpu_baseline` (the reference
compressor, O_ref, single thread on a bounded sample).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "bzip2-opencl_amd")
sys.path.insert(0, PKG)

METRIC = "compress MB/s at -9 (900KB blocks), bit-exact .bz2; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


WORKLOADS = {
    "random": "C2: {mib} MiB random bytes per GPU (torch Philox, seed 0x5EED0001+rank) resident in HBM -> "
              "one .bz2 stream per GPU",
    "text": "C3: {mib} MiB seeded word-Markov text per GPU (synth.text_bytes, seed 0x5EED0002+rank; enwik9 "
            "stand-in) resident in HBM -> one .bz2 stream per GPU",
    "mixed": "C4: {mib} MiB mixed-entropy stream per GPU (synth.mixed_bytes, seed 0x5EED0003+rank, 64 MiB "
             "segments of random/text/runs/ACGT) resident in HBM -> one .bz2 stream per GPU",
}


def ensure_built():
    so = os.path.join(PKG, "bz2mi", "libbz2mi.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, stdout=subprocess.DEVNULL)


TRAFFIC_PROFILE = os.path.join(REPO, "profiles", "r01_traffic.json")


def stage_traffic(args, stage):
    """HBM-side bytes per launch of `stage` from the committed rocprofv3 --pmc
    passes of this same command (tools/round_profile.sh -> tools/traffic.py:
    FETCH_SIZE x2 per the gfx950 note of MI355X_MICROARCH.md, + WRITE_SIZE).
    Only for the workload those passes ran (C2 at the default level/p/unit)."""
    if args.data != "random" or args.mib != 1024 or args.level != 9 or args.parallel != 10 or args.unit != 10000:
        return None, None
    try:
        with open(TRAFFIC_PROFILE) as f:
            prof = json.load(f)
        return int(prof["stages"][stage]["traffic_bytes"]), os.path.relpath(TRAFFIC_PROFILE, REPO)
    except (OSError, KeyError, ValueError):
        return None, None


def cpu_baseline(sample_bytes: int) -> dict:
    """Reference compressor (O_ref = the reference's own kernel.cpp + host code,
    oracle/_ref/liboref.so) or, where it was not built, the C restatement
    cpu_ref; one thread, bounded sample of the same workload."""
    import numpy as np
    from bz2mi import synth
    data = synth.random_bytes(sample_bytes).tobytes()
    oref = os.path.join(REPO, "oracle", "_ref", "liboref.so")
    cref = os.path.join(REPO, "oracle", "_build", "libcpuref.so")
    if os.path.exists(oref):
        L = ctypes.CDLL(oref)
        L.oref_compress.restype = ctypes.c_longlong
        L.oref_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_char_p, ctypes.c_size_t]
        cap = len(data) * 2 + (1 << 20)
        out = ctypes.create_string_buffer(cap)
        t0 = time.perf_counter()
        n = L.oref_compress(data, len(data), 9, 10, 10000, out, cap)
        dt = time.perf_counter() - t0
        kind = "reference"
        label = "O_ref (reference kernel.cpp + BlockCompressor/BitOutputStream compiled for the host, serial)"
    elif os.path.exists(cref):
        L = ctypes.CDLL(cref)
        L.cpuref_compress.restype = ctypes.c_longlong
        L.cpuref_bound.restype = ctypes.c_size_t
        cap = L.cpuref_bound(ctypes.c_size_t(len(data)), 9, 10000)
        out = ctypes.create_string_buffer(cap)
        t0 = time.perf_counter()
        n = L.cpuref_compress(data, ctypes.c_size_t(len(data)), 9, 10, 10000, out, ctypes.c_size_t(cap), 1)
        dt = time.perf_counter() - t0
        kind = "port"
        label = "cpu_ref (oracle/cpu_ref.c restatement)"
    else:
        return None
    if n < 0:
        return None
    return {"value": round(len(data) / dt / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": kind,
            "sample": f"{len(data) >> 20} MiB of the same random-byte workload at -9, p=10, one thread: {label}",
            "seconds": round(dt, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mib", type=int, default=1024, help="input MiB per GPU (default 1 GiB)")
    ap.add_argument("--level", type=int, default=9)
    ap.add_argument("--parallel", type=int, default=10)
    ap.add_argument("--unit", type=int, default=10000, help="block unit: 10000 (reference) or 100000 (900 KB)")
    ap.add_argument("--cpu-sample-mib", type=int, default=96)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--mode", choices=["compress", "decompress"], default="compress",
                    help="compress = the bench line (BASELINE metric); decompress = configs[4]: device "
                         "decompression of the stream this run compresses (output MB/s)")
    ap.add_argument("--data", choices=["random", "text", "mixed"], default="random",
                    help="random = C2 (the bench line); text = C3 stand-in (seeded word Markov text, enwik9 is "
                         "not available offline); mixed = C4 (rotating random/text/runs/ACGT segments)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    ensure_built()
    import bz2mi

    n = args.mib << 20
    dev = torch.device("cuda", local)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0001 + rank)
    if args.data == "random":
        x = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev, generator=g)
    else:
        from bz2mi import synth
        gen = synth.text_bytes if args.data == "text" else synth.mixed_bytes
        x = torch.from_numpy(gen(n, (synth.SEED_TEXT if args.data == "text" else synth.SEED_MIXED) + rank)).to(dev)
    cap = bz2mi.compress_bound(n, args.level, args.unit)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    ctx = bz2mi.Context(args.level, args.parallel, args.unit, device=local)
    ctx.stats()  # enable volume collection

    def step():
        return ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)

    if args.mode == "decompress":
        return bench_decompress(args, ctx, x, n, out, cap, world, rank, dev)

    for _ in range(args.warmup):
        out_len = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    stage_sum = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out_len = step()
        for k, v in ctx.timings().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    stats = ctx.stats()

    # correctness: the stream decodes back to the input (prefix check with the
    # host bzip2 decoder; full-size parity lives in tests/)
    verified = None
    if not args.no_verify and rank == 0:
        import bz2
        head = out[: min(out_len, 4 << 20)].cpu().numpy().tobytes()
        d = bz2.BZ2Decompressor()
        try:
            got = d.decompress(head, max_length=2 << 20)
            verified = bool(got == x[: len(got)].cpu().numpy().tobytes() and len(got) > 0)
        except Exception:
            verified = False

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    steps = args.steps
    ms_step = dt / steps * 1e3
    value = world * n * steps / dt / 1e6
    avg = {k: v / steps for k, v in stage_sum.items()}
    # algorithmic bytes per launch of each stage (DESIGN.md "Roofline")
    rle1 = stats["rle1_bytes"]
    syms = stats["mtf_symbols"]
    payload = stats["payload_bits"] // 8
    nb = stats["blocks"]
    alg = {
        "front": 2 * n + rle1,                       # read input twice (scan + emission), write RLE1 blocks
        "bwt": 2 * rle1 + 4 * nb,                    # read block, write BWT (+ origPtr)
        "mtf": rle1 + 2 * syms + 258 * 4 * nb,       # read BWT, write u16 symbols + histogram
        "huffman": 2 * syms + payload,               # read symbols, write payload
        "assemble": payload + out_len,               # read payload, write stream
    }
    dom = max((k for k in alg if avg.get(k, 0) > 0), key=lambda k: avg[k])
    achieved = alg[dom] / (avg[dom] * 1e-3) / 1e9
    traffic, tsrc = stage_traffic(args, dom)
    roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
            "algorithmic_bytes": int(alg[dom]), "avg_ms": round(avg[dom], 3),
            "pipeline_GBps": round((n + out_len) / (ms_step * 1e-3) / 1e9, 2),
            "stage_ms": {k: round(v, 3) for k, v in avg.items()}}
    cpu = None if args.no_cpu else cpu_baseline(args.cpu_sample_mib << 20)
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": WORKLOADS[args.data].format(mib=args.mib),
                   "level": args.level, "block_size": args.level * args.unit, "parallel_blocks": args.parallel,
                   "input_bytes_per_gpu": n, "output_bytes": int(out_len), "ratio": round(out_len / n, 5),
                   "blocks": nb, "parallelism": f"dp{world} (independent streams)", "decode_check": verified},
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_decompress(args, ctx, x, n, out, cap, world, rank, dev):
    """configs[4]: decompression on the device of the .bz2 this run produced
    (bz2mi's own stream: the reference decoder's block-size limit).
    One step = the whole stream decoded (candidate scan, Huffman/MTF/RLE2,
    inverse BWT, RLE1 + CRC checks); value = decompressed MB/s."""
    import torch
    import torch.distributed as dist
    import bz2mi
    zlen = ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)
    y = torch.empty(n, dtype=torch.uint8, device=dev)
    d = bz2mi.Decompressor(args.unit)
    for _ in range(args.warmup):
        d.decompress_device(out.data_ptr(), zlen, y.data_ptr(), n)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    stage = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        got = d.decompress_device(out.data_ptr(), zlen, y.data_ptr(), n)
        for k, v in d.timings().items():
            stage[k] = stage.get(k, 0.0) + v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ok = bool(got == n and torch.equal(x, y))
    if rank == 0:
        line = {
            "metric": "decompress MB/s (.bz2 from this run, -9), output bytes", "value": round(world * n * args.steps / dt / 1e6, 2),
            "unit": "MB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "configs[4] stand-in: " + WORKLOADS[args.data].format(mib=args.mib),
                       "compressed_bytes": int(zlen), "round_trip_equal": ok},
            "stage_ms": {k: round(v / args.steps, 3) for k, v in stage.items()},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
