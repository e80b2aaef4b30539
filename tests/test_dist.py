"""N>1 path of bench.py on the CPU: world_size-2 gloo over 127.0.0.1.

bench.py shards streams across ranks with no data-path collective
(SURVEY.md §8e): contiguous ranges from shard_streams(), MAX of the timed
region and SUM of the counters through reduce_stats().  Here each rank
demodulates its shard with the oracle and the result must equal the
single-process run; the GPU leg of the same code is the driver's N-GPU bench.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import common as K
import oracle as O

TOTAL = 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _signals(lo, hi):
    return [K.stream_signal(1000 + g, sps=8, span=8, n_bits=600) for g in range(lo, hi)]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = bench.shard_streams(TOTAL, rank, world)
        bits = [K.oracle_for(8, 8).DeModulate(x) for x in _signals(lo, hi)]
        nbits = sum(len(b) for b in bits)
        t, (c_bits, c_streams) = bench.reduce_stats(0.5 + rank, [nbits, hi - lo])
        gathered = [None] * world
        dist.all_gather_object(gathered, (lo, bits))
        if rank == 0:
            q.put((t, c_bits, c_streams, gathered))
    finally:
        dist.destroy_process_group()


def test_shard_streams_partition():
    for total in (1, 7, 256, 32768):
        for world in (1, 2, 3, 8):
            r = [bench.shard_streams(total, k, world) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            assert max(h - l for l, h in r) - min(h - l for l, h in r) <= 1


def test_reduce_stats_single_process_passthrough():
    assert bench.reduce_stats(1.25, [3, 4]) == (1.25, [3, 4])


def test_two_rank_gloo_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        t, c_bits, c_streams, gathered = q.get(timeout=180)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert t == 1.5                       # MAX over ranks
    assert c_streams == TOTAL             # SUM over ranks
    ref = [K.oracle_for(8, 8).DeModulate(x) for x in _signals(0, TOTAL)]
    assert c_bits == sum(len(b) for b in ref)
    merged = [b for _, bits in sorted(gathered) for b in bits]
    assert merged == ref


def test_ber_windowed_realignment_counts_slips_not_errors():
    rng = np.random.default_rng(3)
    tx = rng.integers(0, 2, 40000).astype(np.uint8)
    # decoded stream: drops the first dibit, one symbol slip (2 bits) at 20000,
    # and 5 isolated bit errors
    rx = np.concatenate([tx[2:20000], tx[20002:]])
    for k in (9000, 12001, 15007, 25003, 30011):
        rx[k] ^= 1
    to_t = lambda a: torch.from_numpy(np.packbits(a)[None, :].copy())  # noqa: E731
    e, tot, lost, slips = bench.ber_after_lock(to_t(rx), torch.tensor([rx.size]), to_t(tx), 1)
    assert slips == 1
    assert e <= 5 and e >= 5 - lost    # an error inside a key loses that window instead
    assert tot > 25000
