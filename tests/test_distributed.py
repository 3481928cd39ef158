"""Multi-process sharding on CPU (gloo, world size 2): every rank compresses
its own seeded object (cpu_ref stands in for the device here), the streams are
gathered in rank order, and the multi-stream result decodes to the
concatenation of the objects."""
from __future__ import annotations

import bz2
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import CpuRef


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bz2mi import dist as bdist
    from bz2mi import synth
    data = synth.text_bytes(200_000 + 77_777 * rank, bdist.object_seed(0x5EED0002, rank)).tobytes()
    stream = CpuRef().compress(data, 9, 10)
    got = bdist.gather_streams(torch.frombuffer(bytearray(stream), dtype=torch.uint8))
    datas = [None] * world
    dist.all_gather_object(datas, data)
    if rank == 0:
        combined = bdist.concat_streams(got)
        q.put(bz2.decompress(combined) == b"".join(datas) and len(got) == world)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_two_ranks_gather_streams():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert ok
    assert all(p.exitcode == 0 for p in procs)
