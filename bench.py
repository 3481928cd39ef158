#!/usr/bin/env python3
"""bench.py -- compress throughput of the MI355X bzip2 path (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 1 GiB of random
bytes resident in HBM, compressed at -9 with the reference's block size
(S = 9 x 10,000 = 90,000 bytes, Config.hpp:30) and parallel count p = 10, to a
complete .bz2 stream in HBM.  One step = one whole stream: device RLE1 front
end + block split + CRCs, BWT, MTF/RLE2, seed carry-over, Huffman + packing,
stream assembly.  Multi-GPU (--gpus N: one process per GPU, self-launched
through torch.distributed.run when not started by it): ONE logical stream of
N x 1 GiB, cut into units interleaved over the ranks, compressed with the unit
protocol of bz2mi.shard (chain token, seed-sum all-gather, bit-offset scan;
SURVEY.md section 8(e)) into the same bytes one device would write -> weak
scaling; timing is the max over ranks.

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
    "realtext": "C3: {mib} MiB enwik9-like text per GPU (synth.realtext_bytes, seed 0x5EED0004+rank: mixed case, "
                "digits, MediaWiki/XML markup and page headers, UTF-8 words, repeated 0.2-20 KB passages; ~150 "
                "distinct bytes per 90 KB block; enwik9 itself is not available offline) resident in HBM -> one .bz2 "
                "stream per GPU",
    "mixed": "C4: {mib} MiB mixed-entropy stream per GPU (synth.mixed_bytes, seed 0x5EED0003+rank, 64 MiB "
             "segments of random/text/runs/ACGT) resident in HBM -> one .bz2 stream per GPU",
}


def ensure_built():
    so = os.path.join(PKG, "bz2mi", "libbz2mi.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, stdout=subprocess.DEVNULL)


# committed rocprofv3 passes of this same command (tools/r5_measure.sh):
# traffic (FETCH_SIZE x2 + WRITE_SIZE, tools/traffic.py), issue (SQ/GRBM
# counters, tools/issue.py) and kernel stats; each file records the sha256 of
# the library it was measured with, and a file from another build is not used
PROFILE_ROUND = "r06"
TRAFFIC_PROFILE = os.path.join(REPO, "profiles", PROFILE_ROUND + "_traffic_{name}.json")
ISSUE_PROFILE = os.path.join(REPO, "profiles", PROFILE_ROUND + "_issue_{name}.json")
KSTATS_PROFILE = "profiles/" + PROFILE_ROUND + "_kernel_stats_{name}.csv"
# the kernels of each timed stage (bz2mi_compress_device, csrc/api.hip)
STAGE_KERNELS = {
    "front": "fe_summary/runscan/costscan/dmap/chain/resolve (scans + block chain) and fe_rle1_kernel",
    "bwt": "90 KB blocks: bwt_block_kernel x2 (mode 0: first-byte scatter + batch sorts; mode 1: blocks the text "
           "kernel hands back), bwt_text_kernel, bwt_wlevel/level/block_small kernels, bwt_tie_kernel x6, "
           "bwt_double_kernel; 900 KB blocks: bwt_bucket/bigbucket/wlevel/level/small kernels, bwt_tie_kernel x3, "
           "dbl_* (grid-wide prefix doubling)",
    "mtf": "mtf_kernel<G>",
    "huffman": "huffman_kernel",
    "assemble": "offsets_dev_kernel, assemble_dev_kernel, advance_kernel",
}


def lib_sha16() -> str | None:
    """sha256 (16 hex digits) of the library this process loads."""
    import hashlib
    path = os.environ.get("BZ2MI_LIBRARY") or os.path.join(PKG, "bz2mi", "libbz2mi.so")
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def profile_name(data: str, unit: int) -> str:
    return data + ("900k" if unit == 100000 else "")


def _profile(path: str):
    """A committed profile of this build: (json, relpath, None) or (None, relpath, why)."""
    rel = os.path.relpath(path, REPO)
    try:
        with open(path) as f:
            prof = json.load(f)
    except (OSError, ValueError):
        return None, rel, "no profile"
    sha = lib_sha16()
    if prof.get("lib_sha16") != sha:
        return None, rel, f"measured with library {prof.get('lib_sha16')}, this run loads {sha}"
    return prof, rel, None


def default_shape(args) -> bool:
    return args.mib == 1024 and args.level == 9 and args.parallel == 10


def stage_traffic(args, stage, unit):
    """HBM-side bytes per launch of `stage` from the committed rocprofv3 --pmc
    passes of this same command and build (FETCH_SIZE x2 per the gfx950 note of
    MI355X_MICROARCH.md, + WRITE_SIZE).  Only for the workloads those passes
    ran (1 GiB at -9, p = 10)."""
    if not default_shape(args):
        return None, None, "not a profiled workload"
    prof, rel, why = _profile(TRAFFIC_PROFILE.format(name=profile_name(args.data, unit)))
    if prof is None:
        return None, rel, why
    try:
        return int(prof["stages"][stage]["traffic_bytes"]), rel, None
    except (KeyError, ValueError):
        return None, rel, "stage missing"


ISSUE_PREFIX = {"front": ("fe_",), "bwt": ("bwt_", "dbl_"), "mtf": ("mtf_kernel",), "huffman": ("huffman_kernel",),
                "assemble": ("assemble", "offsets_dev", "advance")}


def stage_issue(args, stage, unit):
    """VALU issue utilisation and LDS bank-conflict share of the stage's
    kernels, from the committed SQ/GRBM --pmc pass of this same command and
    build (tools/issue.py); kernels taking <2% of the stage's profiled time
    are left out."""
    if not default_shape(args):
        return None
    prof, rel, why = _profile(ISSUE_PROFILE.format(name=profile_name(args.data, unit)))
    if prof is None:
        return {"source": rel, "unavailable": why}
    ks = {k: v for k, v in prof["kernels"].items() if k.startswith(ISSUE_PREFIX[stage])}
    tot = sum(v["ms_total"] for v in ks.values()) or 1.0
    keep = {k: {a: v[a] for a in ("valu_issue_frac", "lds_bank_conflict_frac", "salu_per_valu", "eff_clock_GHz")
                if a in v} | {"time_share": round(v["ms_total"] / tot, 3)}
            for k, v in ks.items() if v["ms_total"] >= 0.02 * tot}
    return {"source": rel, "kernels": keep,
            "what": "SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE/8): the share of SIMD issue "
                    "slots the kernel's VALU stream used; SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE"}


def roofline(args, unit, n, stats, avg, out_len, ms_step):
    """The dominant stage against the HBM roofline: algorithmic bytes per
    launch (DESIGN.md "Roofline") / its HIP-event time, the committed traffic
    and issue passes of this build, the pipeline rate."""
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
    traffic, tsrc, why = stage_traffic(args, dom, unit)
    return {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
            "traffic_unavailable": why,
            "algorithmic_bytes": int(alg[dom]), "avg_ms": round(avg[dom], 3),
            "stage_kernels": STAGE_KERNELS.get(dom),
            "issue": stage_issue(args, dom, unit),
            "lib_sha16": lib_sha16(),
            "what": "HIP events around the stage's launches on the stream they run on, per step; the stage is "
                    "the kernels listed (their rocprofv3 durations sum to avg_ms: "
                    + KSTATS_PROFILE.format(name=profile_name(args.data, unit)) + ")",
            "pipeline_GBps": round((n + out_len) / (ms_step * 1e-3) / 1e9, 2),
            "stage_ms": {k: round(v, 3) for k, v in avg.items()}}


def host_cpu() -> dict:
    """Host CPU model and the cores this process may use: the GPU box gives a
    1-GPU job a share of the machine (OMP_NUM_THREADS / MAX_JOBS = 16 there,
    while os.sched_getaffinity lists every core of the host), so the parallel
    baseline uses that share, capped by the affinity mask."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    share = 0
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        try:
            share = max(share, int(os.environ.get(var, "0")))
        except ValueError:
            pass
    used = max(1, min(avail, share if share > 0 else avail))
    return {"model": model, "cores_in_affinity_mask": avail, "job_cpu_share": share or None,
            "cores_used_parallel": used}


def cpu_baseline(sample_bytes: int) -> dict:
    """Reference compressor (O_ref = the reference's own kernel.cpp + host code,
    oracle/_ref/liboref.so) or, where it was not built, the C restatement
    cpu_ref; one thread, bounded sample of the same workload.  Context in the
    same run: cpu_ref on all usable cores (block-parallel, bit-identical output)
    and libbz2 1.0.8 at -9 (bzip2's own 900 KB blocks, different bytes)."""
    import bz2
    from bz2mi import synth
    data = synth.random_bytes(sample_bytes).tobytes()
    oref = os.path.join(REPO, "oracle", "_ref", "liboref.so")
    cref = os.path.join(REPO, "oracle", "_build", "libcpuref.so")
    cpu = host_cpu()
    res = None
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
        if n >= 0:
            res = {"value": round(len(data) / dt / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "reference",
                   "sample": f"{len(data) >> 20} MiB of the same random-byte workload at -9, p=10, one thread: "
                             "O_ref (reference kernel.cpp + BlockCompressor/BitOutputStream compiled for the host, "
                             "serial)", "seconds": round(dt, 2)}
    if os.path.exists(cref):
        L = ctypes.CDLL(cref)
        L.cpuref_compress.restype = ctypes.c_longlong
        L.cpuref_bound.restype = ctypes.c_size_t
        cap = L.cpuref_bound(ctypes.c_size_t(len(data)), 9, 10000)
        out = ctypes.create_string_buffer(cap)
        if res is None:
            t0 = time.perf_counter()
            n = L.cpuref_compress(data, ctypes.c_size_t(len(data)), 9, 10, 10000, out, ctypes.c_size_t(cap), 1)
            dt = time.perf_counter() - t0
            if n >= 0:
                res = {"value": round(len(data) / dt / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "port",
                       "sample": f"{len(data) >> 20} MiB of the same random-byte workload at -9, p=10, one "
                                 "thread: cpu_ref (oracle/cpu_ref.c restatement)", "seconds": round(dt, 2)}
        th = cpu["cores_used_parallel"]
        t0 = time.perf_counter()
        n = L.cpuref_compress(data, ctypes.c_size_t(len(data)), 9, 10, 10000, out, ctypes.c_size_t(cap), th)
        dt = time.perf_counter() - t0
        if res is not None and n >= 0:
            res["all_cores"] = {"value": round(len(data) / dt / 1e6, 3), "unit": "MB/s", "threads": th,
                                "what": "cpu_ref block-parallel on a pthread pool, same bytes as O_ref, on every "
                                        "core this job may use (host_cpu: the job's CPU share)"}
    if res is None:
        return None
    sub = data[: min(len(data), 32 << 20)]
    t0 = time.perf_counter()
    bz2.compress(sub, 9)
    dt = time.perf_counter() - t0
    res["bzip2_9"] = {"value": round(len(sub) / dt / 1e6, 3), "unit": "MB/s", "threads": 1,
                      "what": f"libbz2 1.0.8 -9 (900 KB blocks) on {len(sub) >> 20} MiB of the sample (context only)"}
    res["host_cpu"] = cpu
    return res


def reference_gpu(sample_bytes: int) -> dict | None:
    """The reference itself on this GPU: its app.cpp + kernel.cpp, unmodified
    (oracle/_ref/ref_app, built from /root/reference), compressing a file of
    random bytes through the ROCm OpenCL runtime at -9 with its thesis setting
    p = 1024 (default p = 10 leaves 10 lanes busy).  Process wall time.
    Its Huffman tables differ from O_ref's (hazard H3, tests/test_refgpu.py);
    the stream is checked to decode."""
    import bz2
    import tempfile
    from bz2mi import synth
    app = os.path.join(REPO, "oracle", "_ref", "ref_app")
    if not os.path.exists(app):
        return None
    data = synth.random_bytes(sample_bytes, 0x5EED2002).tobytes()
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        f = os.path.join(d, "in.bin")
        with open(f, "wb") as h:
            h.write(data)
        t0 = time.perf_counter()
        r = subprocess.run([app, f, "-k", "-s", "9", "-p", "1024"], capture_output=True, timeout=300)
        dt = time.perf_counter() - t0
        if r.returncode != 0:
            return None
        with open(f + ".bz2", "rb") as h:
            z = h.read()
    ok = bz2.decompress(z) == data
    return {"value": round(len(data) / dt / 1e6, 3), "unit": "MB/s", "seconds": round(dt, 2),
            "sample": f"{len(data) >> 20} MiB random bytes, app.cpp -s 9 -p 1024 (file -> file, OpenCL on this GPU)",
            "decodes": ok}


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
    ap.add_argument("--no-900k", action="store_true", help="skip the 900 KB-mode measurement beside the line")
    ap.add_argument("--no-units", action="store_true",
                    help="N = 1: skip the unit-protocol line (4 units, the code N > 1 times) beside the line")
    ap.add_argument("--mode", choices=["compress", "decompress", "e2e"], default="compress",
                    help="compress = the bench line (BASELINE metric); decompress = configs[4]: device "
                         "decompression of the stream this run compresses (output MB/s); e2e = file -> file "
                         "through the reference's unmodified app.cpp built against the mirror headers")
    ap.add_argument("--data", choices=["random", "text", "realtext", "mixed"], default="random",
                    help="random = C2 (the bench line); realtext = C3 stand-in (enwik9-like: ~150 distinct bytes "
                         "per block, markup, UTF-8, long repeats; enwik9 is not available offline); text = 27-symbol "
                         "word Markov text; mixed = C4 (rotating random/text/runs/ACGT segments)")
    ap.add_argument("--units-per-gpu", type=int, default=None,
                    help="units of the logical stream per rank (interleaved over the ranks); N > 1 default 4; "
                         "given at N = 1, the unit protocol runs on the one device (the base of a 1 -> N curve)")
    ap.add_argument("--gather", choices=["none", "rank0"], default="rank0",
                    help="N > 1: rank0 (default) = the ordered RCCL gather of the stream onto rank 0 is inside "
                         "the timed step, so the value is a whole .bz2 on one rank; none = the stream ends "
                         "distributed (each rank holds its units' final bytes), the gather timed once after")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: relaunch under torch.distributed.run before any GPU call
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or args.units_per_gpu is not None:
        if args.units_per_gpu is None:
            args.units_per_gpu = 4
        return bench_units(args, world)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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
        if args.data == "realtext":
            host = synth.realtext_bytes(n, synth.SEED_REALTEXT + rank, threads=host_cpu()["cores_used_parallel"])
        else:
            gen = synth.text_bytes if args.data == "text" else synth.mixed_bytes
            host = gen(n, (synth.SEED_TEXT if args.data == "text" else synth.SEED_MIXED) + rank)
        x = torch.from_numpy(host).to(dev)
        del host
    cap = bz2mi.compress_bound(n, args.level, args.unit)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    ctx = bz2mi.Context(args.level, args.parallel, args.unit, device=local)
    ctx.stats()  # enable volume collection

    def step():
        return ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)

    if args.mode == "decompress":
        return bench_decompress(args, ctx, x, n, out, cap, world, rank, dev)
    if args.mode == "e2e":
        return bench_e2e(args, ctx, x, n, out, cap)

    for _ in range(args.warmup):
        out_len = step()
    torch.cuda.synchronize()
    stage_sum = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out_len = step()
        for k, v in ctx.timings().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stats = ctx.stats()

    # correctness: the stream decodes back to the input (prefix check with the
    # host bzip2 decoder; full-size parity lives in tests/)
    verified = None
    if not args.no_verify:
        import bz2
        head = out[: min(out_len, 4 << 20)].cpu().numpy().tobytes()
        d = bz2.BZ2Decompressor()
        try:
            got = d.decompress(head, max_length=2 << 20)
            verified = bool(got == x[: len(got)].cpu().numpy().tobytes() and len(got) > 0)
        except Exception:
            verified = False

    steps = args.steps
    ms_step = dt / steps * 1e3
    value = world * n * steps / dt / 1e6
    avg = {k: v / steps for k, v in stage_sum.items()}
    nb = stats["blocks"]
    roof = roofline(args, args.unit, n, stats, avg, out_len, ms_step)
    # the metric's literal wording, "900KB blocks": the same input at -9 in the
    # 900 KB mode (unit 100000, S = 900,000; O_ref900 pins),
    # timed the same way right after the line's own steps
    mode900 = None
    # one context at a time: each holds its own streams, and two contexts'
    # streams share the device's hardware queues (GPU_MAX_HW_QUEUES = 4), which
    # serialises the second context's pipelined stages
    del out
    ctx.close()
    torch.cuda.empty_cache()
    if not args.no_900k and args.unit == 10000 and args.level == 9:
        ctx9 = bz2mi.Context(args.level, args.parallel, 100000, device=local)
        ctx9.stats()
        cap9 = bz2mi.compress_bound(n, args.level, 100000)
        out9 = torch.empty(cap9, dtype=torch.uint8, device=dev)
        for _ in range(max(1, args.warmup)):
            z9 = ctx9.compress_device(x.data_ptr(), n, out9.data_ptr(), cap9)
        torch.cuda.synchronize()
        st9 = {}
        t9 = time.perf_counter()
        for _ in range(args.steps):
            z9 = ctx9.compress_device(x.data_ptr(), n, out9.data_ptr(), cap9)
            for k, v in ctx9.timings().items():
                st9[k] = st9.get(k, 0.0) + v
        torch.cuda.synchronize()
        dt9 = time.perf_counter() - t9
        ok9 = None
        if not args.no_verify:
            import bz2
            head9 = out9[: min(z9, 4 << 20)].cpu().numpy().tobytes()
            try:
                got9 = bz2.BZ2Decompressor().decompress(head9, max_length=2 << 20)
                ok9 = bool(len(got9) > 0 and got9 == x[: len(got9)].cpu().numpy().tobytes())
            except Exception:
                ok9 = False
        stats9 = ctx9.stats()
        ms9 = dt9 / args.steps * 1e3
        mode900 = {"value": round(n * args.steps / dt9 / 1e6, 2), "unit": "MB/s",
                   "ms_per_step": round(ms9, 3), "block_size": args.level * 100000,
                   "blocks": stats9["blocks"], "output_bytes": int(z9), "decode_check": ok9,
                   "roofline": roofline(args, 100000, n, stats9, {k: v / args.steps for k, v in st9.items()}, z9, ms9),
                   "what": "the same input and steps at -9 in the 900 KB mode (unit 100000; O_ref900 pins)"}
        del out9
        ctx9.close()
    # the code the N > 1 lines time, at N = 1: the same workload as 4 units of
    # one logical stream through bz2mi.shard (the base of the 1 -> N curve)
    units_n1 = None
    if not args.no_units and world == 1 and args.mode == "compress":
        import copy
        a2 = copy.copy(args)
        a2.units_per_gpu, a2.no_cpu = 4, True
        u = bench_units(a2, 1, emit=False)
        units_n1 = {k: u[k] for k in ("value", "ms_per_step")}
        units_n1.update({"units": 4, "decode_check": u["config"]["decode_check"],
                         "gather_in_step": u["config"]["gather_in_step"],
                         "stage_ms": u["roofline"]["stage_ms_rank0"],
                         "what": "the same data shape as 4 units of 256 MiB through the unit protocol (chain token, "
                                 "seed-sum token, bit offsets, assembly, ordered gather) on this one device: the "
                                 "code the N > 1 lines time"})
    cpu = None if args.no_cpu else cpu_baseline(args.cpu_sample_mib << 20)
    refgpu = None if args.no_cpu else reference_gpu(64 << 20)
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": WORKLOADS[args.data].format(mib=args.mib),
                   "level": args.level, "block_size": args.level * args.unit, "parallel_blocks": args.parallel,
                   "input_bytes_per_gpu": n, "output_bytes": int(out_len), "ratio": round(out_len / n, 5),
                   "blocks": nb, "parallelism": "dp1 (one stream, one device call)", "decode_check": verified},
        "roofline": roof,
        "mode_900k": mode900,
        "unit_protocol_n1": units_n1,
        "cpu_baseline": cpu,
        "reference_on_this_gpu": refgpu,
    }
    print(json.dumps(line), flush=True)


def unit_bytes(args, g: int, U: int, dev):
    """Unit g of the logical stream (U bytes) on `dev`: random = torch Philox
    with seed 0x5EED0001 + g; text = word-Markov text with seed 0x5EED0002 + g;
    mixed = the C4 stream of 64 MiB segments (unit g = segments g*U/64Mi ...)."""
    import torch
    from bz2mi import synth
    if args.data == "random":
        gen = torch.Generator(device=dev)
        gen.manual_seed(synth.SEED_RANDOM + g)
        return torch.randint(0, 256, (U,), dtype=torch.uint8, device=dev, generator=gen)
    if args.data == "text":
        return torch.from_numpy(synth.text_bytes(U, synth.SEED_TEXT + g)).to(dev)
    if args.data == "realtext":
        return torch.from_numpy(synth.realtext_bytes(U, synth.SEED_REALTEXT + g, threads=8)).to(dev)
    seg = 64 << 20
    assert U % seg == 0, "mixed units are whole 64 MiB segments"
    return torch.from_numpy(synth.mixed_bytes(U, synth.SEED_MIXED, seg, first_segment=g * (U // seg))).to(dev)


def bench_units(args, world: int, emit: bool = True):
    """N ranks, one logical stream (SURVEY.md section 8(e), config C4's layout):
    world x units-per-gpu units of U = mib/units-per-gpu MiB, unit g on rank
    g mod world; every unit buffer = its bytes + the tail halo (the bytes of the
    following units, bz2mi_unit_halo of them or up to the stream end).  One
    step = the whole stream through bz2mi.shard: front scans, chain (token in
    stream order), seed-sum all-gather, Huffman, bit-offset scan, assembly and
    boundary settling; with --gather rank0 also the ordered RCCL gather onto
    rank 0.  world == 1 (--units-per-gpu at --gpus 1): the same protocol on one
    device, the base of a 1 -> N curve that times the same code at every N.
    After the timed steps the whole stream is gathered onto rank 0, decoded on
    the device and compared with every unit's input."""
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BZ2MI_SHARE_GPU=1: rehearsal of the N-rank protocol with every rank on
    # cuda:0 (one-GPU box): gloo everywhere, pieces gathered over the host
    share = os.environ.get("BZ2MI_SHARE_GPU") == "1"
    if share:
        local = 0
    dev = torch.device("cuda", local)
    torch.cuda.set_device(local)
    ctl = None
    if world > 1:
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        ctl = dist.new_group(backend="gloo")

    def barrier():
        if world > 1:
            dist.barrier()

    ensure_built()
    import bz2mi
    from bz2mi import shard
    K = args.units_per_gpu
    n = args.mib << 20
    U = n // K
    total = world * K
    owners = shard.interleaved_owners(total, world)
    H = bz2mi.unit_halo(args.level, args.unit)
    ctx = bz2mi.Context(args.level, args.parallel, args.unit, device=local)
    mine = [g for g in range(total) if owners[g] == rank]
    bufs, halos, ends, units = {}, {}, {}, {}
    for g in mine:
        # tail halo: the bytes of the following units until H of them or the stream end
        parts = [unit_bytes(args, g, U, dev)]
        got, h = 0, g + 1
        while got < H and h < total:
            nxt = unit_bytes(args, h, U, dev)[: H - got]
            parts.append(nxt)
            got += int(nxt.numel())
            h += 1
        bufs[g] = torch.cat(parts)
        halos[g] = got
        ends[g] = got < H  # the halo reaches the end of the stream
        del parts
        units[g] = shard.DeviceUnit(ctx, dev)
    torch.cuda.synchronize()
    out0 = None
    if rank == 0:
        bound = bz2mi.compress_bound(n * world, args.level, args.unit)
        out0 = torch.empty(bound, dtype=torch.uint8, device=dev)

    # BZ2MI_UNIT_TRACE=<prefix>: every rank writes the host timeline of its
    # last step (chain token arrivals, chain ends, seed rounds, encodes) to
    # <prefix>.<rank>.json (tools/unit_hops.py: per-hop latency, critical path)
    trace_path = os.environ.get("BZ2MI_UNIT_TRACE")
    trace = [] if trace_path else None

    def step(gather: bool):
        if trace is not None:
            trace.clear()
            trace.append(("step", -1, time.perf_counter()))
        for g in mine:
            units[g].begin(bufs[g], U, halos[g], ends[g])
        # one rank: every unit assembled in place in the stream buffer
        lay = shard.compress_units(units, owners, args.parallel, args.level, group=ctl,
                                   out=out0 if world == 1 else None, trace=trace,
                                   seeds=os.environ.get("BZ2MI_SEEDS", "rounds"))
        if trace is not None:
            torch.cuda.synchronize()
            trace.append(("end", -1, time.perf_counter()))
        settled = shard.settle(lay, ctl)
        if gather:
            shard.gather_stream_device(lay, settled, out0, args.level, dst=0)
        return lay, settled

    gather_in = args.gather == "rank0" and not share
    for _ in range(args.warmup):
        step(gather_in)
    torch.cuda.synchronize()
    barrier()
    stage = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        lay, settled = step(gather_in)
        for g in mine:
            for k, v in units[g].timings().items():
                stage[k] = stage.get(k, 0.0) + v
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if trace is not None:
        with open(f"{trace_path}.{rank}.json", "w") as f:
            json.dump({"rank": rank, "world": world, "units": total, "unit_bytes": U, "owners": owners,
                       "events": trace}, f)
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device="cpu" if share else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    # the ordered gather onto rank 0, timed once (outside the steps unless --gather rank0)
    gather_ms = None
    if not share:
        torch.cuda.synchronize()
        barrier()
        tg = time.perf_counter()
        shard.gather_stream_device(lay, settled, out0, args.level, dst=0)
        torch.cuda.synchronize()
        barrier()
        gather_ms = (time.perf_counter() - tg) * 1e3
    else:  # shared GPU: the pieces travel to rank 0 over the host
        for g in list(lay.pieces):
            t, nb = lay.pieces[g]
            lay.pieces[g] = t[:nb].cpu().numpy().tobytes()
        host_stream = shard.gather_stream_host(lay, args.level, group=ctl)
        if rank == 0:
            out0 = torch.frombuffer(bytearray(host_stream), dtype=torch.uint8).to(dev)
    # the whole stream, checked once: decoded on the device, every unit's bytes compared
    verified = None
    if rank == 0 and not args.no_verify:
        zlen = lay.stream_bytes
        y = torch.empty(n * world, dtype=torch.uint8, device=dev)
        d = bz2mi.Decompressor(args.unit)
        try:
            got = d.decompress_device(out0.data_ptr(), zlen, y.data_ptr(), y.numel())
            verified = got == n * world and all(
                torch.equal(y[g * U:(g + 1) * U], unit_bytes(args, g, U, dev)) for g in range(total))
        except Exception:
            verified = False
        del y
        d.close()
    vol = {"rle1_bytes": 0, "mtf_symbols": 0, "payload_bits": 0, "blocks": 0}
    for g in mine:
        for k, v in units[g].stats().items():
            vol[k] += v
    # rank 0's chains of the last step: speculated units, blocks spliced from
    # a speculation, blocks chained from the entry
    spec_sum = {"speculated_units": 0, "spliced_blocks": 0, "chained_blocks": 0}
    for g in mine:
        ci = units[g].chain_info()
        spec_sum["speculated_units"] += int(ci["speculated"])
        spec_sum["spliced_blocks"] += int(ci["spliced"])
        spec_sum["chained_blocks"] += int(ci["chained"])
    if rank == 0:
        steps = args.steps
        ms_step = dt / steps * 1e3
        tot_in = n * world
        value = tot_in * steps / dt / 1e6
        out_bytes = lay.stream_bytes
        avg = {k: v / steps for k, v in stage.items()}
        # rank 0's units: algorithmic bytes of the dominant device stage (as the N = 1 line)
        alg = {"bwt": 2 * vol["rle1_bytes"] + 4 * vol["blocks"],
               "mtf": vol["rle1_bytes"] + 2 * vol["mtf_symbols"] + 258 * 4 * vol["blocks"],
               "huffman": 2 * vol["mtf_symbols"] + vol["payload_bits"] // 8}
        dom = max((k for k in alg if avg.get(k, 0) > 0), key=lambda k: avg[k])
        achieved = alg[dom] / (avg[dom] * 1e-3) / 1e9
        cpu = None if args.no_cpu else cpu_baseline(args.cpu_sample_mib << 20)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"C4 layout: ONE .bz2 stream of {world} x {args.mib} MiB "
                                   f"({WORKLOAD_DATA[args.data]}), {total} units of {U >> 20} MiB interleaved over "
                                   f"{world} ranks (unit g on rank g mod {world}), blocks sharded by unit; output "
                                   "bit-identical to the one-device stream",
                       "level": args.level, "block_size": args.level * args.unit, "parallel_blocks": args.parallel,
                       "input_bytes_per_gpu": n, "output_bytes": int(out_bytes), "ratio": round(out_bytes / tot_in, 5),
                       "blocks": int(sum(lay.nblocks)), "parallelism": f"dp{world} (block shards of one stream)",
                       "gather_in_step": gather_in, "decode_check": verified,
                       "assembly": "in place in the stream buffer (one rank)" if lay.out is not None
                       else "per-unit pieces, settled and gathered",
                       "speculation": spec_sum,
                       "decode_check_what": "whole stream decoded on rank 0's device, every unit's bytes compared",
                       "shared_gpu_rehearsal": share},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                         "algorithmic_bytes_rank0": int(alg[dom]), "avg_ms_rank0": round(avg[dom], 3),
                         "what": "rank 0's units: the dominant stage's algorithmic bytes / its HIP-event time",
                         "pipeline_GBps": round((tot_in + out_bytes) / (ms_step * 1e-3) / 1e9, 2),
                         "stage_ms_rank0": {k: round(v, 3) for k, v in avg.items()}},
            "gather": None if gather_ms is None else {
                "ms": round(gather_ms, 3), "bytes": int(out_bytes),
                "what": "ordered RCCL point-to-point gather of the settled stream onto rank 0 (once, after the timed "
                        "steps)" if not gather_in else "inside every step",
                "value_with_gather": round(tot_in / ((ms_step + (0 if gather_in else gather_ms)) * 1e-3) / 1e6, 2)},
            "cpu_baseline": cpu,
        }
        if emit:
            print(json.dumps(line), flush=True)
    barrier()
    if world > 1:
        dist.destroy_process_group()
    for g in mine:
        units[g].close()
    ctx.close()
    return line if rank == 0 else None


WORKLOAD_DATA = {"random": "random bytes, unit g seeded 0x5EED0001+g", "text": "word-Markov text, unit g seeded "
                 "0x5EED0002+g", "realtext": "enwik9-like text, unit g seeded 0x5EED0004+g",
                 "mixed": "C4 mixed-entropy segments, seed 0x5EED0003"}


def bench_e2e(args, ctx, x, n, out, cap):
    """End to end, SURVEY.md section 8(d): the reference's app.cpp, unmodified,
    compiled against the mirror OutputStream (raw bytes to the device front end
    in 64 MiB stream units, pinned double buffers), file -> file on the local
    disk: `app_bz2mi <file> -k -s <level> -p <p>`, wall time of the process
    (process start, HIP init, read, compress, write).  The file is checked
    against the device-path stream of the same bytes."""
    import hashlib
    import tempfile
    app = os.path.join(PKG, "build", "app_bz2mi")
    if not os.path.exists(app):
        raise SystemExit("app_bz2mi not built (__graft_entry__.build() in the build container)")
    m = ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)
    want = hashlib.sha256(out[:m].cpu().numpy().tobytes()).hexdigest()
    host = x.cpu().numpy().tobytes()
    times = []
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        src = os.path.join(d, "in.bin")
        with open(src, "wb") as f:
            f.write(host)
        del host
        same = None
        for i in range(args.warmup + args.steps):
            t0 = time.perf_counter()
            subprocess.run([app, src, "-k", "-s", str(args.level), "-p", str(args.parallel)], check=True)
            dt = time.perf_counter() - t0
            with open(src + ".bz2", "rb") as f:
                got = hashlib.sha256(f.read()).hexdigest()
            same = (same is not False) and got == want
            os.unlink(src + ".bz2")
            if i >= args.warmup:
                times.append(dt)
        # where the time goes (tools/e2e_parts.cpp, same file, page cache warm)
        parts = None
        tool = os.path.join(PKG, "build", "e2e_parts")
        if os.path.exists(tool):
            r = subprocess.run([tool, src, str(args.level), str(args.parallel), src + ".parts.bz2"], check=True,
                               capture_output=True, text=True)
            parts = json.loads(r.stdout)
            with open(src + ".parts.bz2", "rb") as f:
                parts["same_bytes"] = hashlib.sha256(f.read()).hexdigest() == want
        open(os.path.join(d, "empty.bin"), "wb").close()
        t1 = time.perf_counter()
        subprocess.run([app, os.path.join(d, "empty.bin"), "-k", "-s", str(args.level), "-p", str(args.parallel)],
                       check=True, capture_output=True)
        t_empty = time.perf_counter() - t1
    t = sum(times) / len(times)
    if parts is not None:
        parts["app_empty_file_s"] = round(t_empty, 4)  # process start + HIP init + an empty stream + teardown
    line = {"metric": "end-to-end compress MB/s (file -> file, unmodified app.cpp on the mirror headers)",
            "value": round(n / t / 1e6, 2), "unit": "MB/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(t * 1e3, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic",
            "config": {"workload": WORKLOADS[args.data].format(mib=args.mib) + " written to a local file",
                       "level": args.level, "parallel_blocks": args.parallel, "unit_bytes": 64 << 20,
                       "same_bytes_as_device_path": bool(same), "seconds": [round(v, 3) for v in times]},
            "breakdown": parts}
    print(json.dumps(line), flush=True)


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
