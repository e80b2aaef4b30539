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
K_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


# ---- the RCCL scatter/gather leg through the same code, gloo ----
SG_STREAMS = 3          # per rank
SG_BITS = 600


def _sg_synth(first, count):
    """Global stream ids -> rows, as Q.synth_generate does on the GPU."""
    sigs = [K.stream_signal(4000 + g, sps=8, span=8, n_bits=SG_BITS) for g in range(first, first + count)]
    n = min(x.size for x in sigs)
    return torch.from_numpy(np.stack([x[:n] for x in sigs]))


def _sg_demod(x):
    bits, nb, _, _ = O.demod_batch_packed(x.numpy(), K.FS, K.FS // 8, n_threads=1,
                                          rrc_alpha=K.ALPHA, rrc_span=8, trig=O.TRIG_PORTABLE)
    return torch.from_numpy(bits), torch.from_numpy(nb)


def _sg_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = _sg_synth(0, 1).shape[1] // 2
        rec, gathered = bench.split_gather(_sg_synth, _sg_demod, SG_STREAMS, n, world, rank,
                                           torch.device("cpu"), host_collectives=True)
        if rank == 0:
            q.put((rec, gathered[0].numpy(), gathered[1].numpy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_split_gather_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sg_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        rec, bits, nb = q.get(timeout=180)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert rec["shards_match_local_synth"] is True
    assert rec["scatter_ms"] >= 0 and rec["gather_ms"] >= 0
    # the gathered rows equal one process demodulating the whole batch
    rb, rnb = _sg_demod(_sg_synth(0, 2 * SG_STREAMS))
    assert np.array_equal(nb, rnb.numpy())
    bad, _ = bench.compare_rows(bits, nb, rb.numpy(), rnb.numpy())
    assert bad == []


def test_compare_rows_masks_the_partial_byte():
    ref = np.array([[0b10110000, 0xFF]], np.uint8)
    got = np.array([[0b10111111, 0x00]], np.uint8)
    assert bench.compare_rows(got, [4], ref, [4])[0] == []
    assert bench.compare_rows(got, [5], ref, [5])[0] == [0]
    assert bench.compare_rows(got, [4], ref, [6])[0] == [0]


def test_pick_streams_covers_the_batch_tail():
    assert bench.pick_streams(100, 500) == list(range(100))
    idx = bench.pick_streams(4096, 200)
    assert idx[:3] == [0, 1, 2] and idx[-64:] == list(range(4032, 4096)) and len(idx) == 200


def test_bench_gpus_flag_must_match_world_size():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(K_ROOT, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in (r.stderr + r.stdout)


def test_steady_state_check_replays_the_call_sequence():
    """bench.steady_state_check feeds the oracle the same buffer `calls` times
    and compares the last call's bits with the handle's rows: rows built from
    that replay pass, one flipped bit is reported by stream."""
    import qpsk_amd as Q
    iq = K.batch_signals(4, seed0=5, sps=8, span=8, n_bits=1500, snr_db=16)
    calls = 3
    rows, nbits = [], []
    for s in range(4):
        d = O.OracleDemod(K.FS, K.FS // 8, K.ALPHA, 8, trig=O.TRIG_LIBM, ring_capacity=4096)
        for _ in range(calls):
            b, _, _ = d.demodulate_ex(iq[s])
        rows.append(np.asarray(Q.pack_bits(b)))
        nbits.append(len(b))
    nb = torch.tensor(nbits, dtype=torch.int64)
    bits = torch.zeros((4, max(r.size for r in rows) + 8), dtype=torch.uint8)
    for s, r in enumerate(rows):
        bits[s, : r.size] = torch.from_numpy(r)
    cfg = dict(bench.CONFIGS["c2"])
    assert bench.steady_state_check(torch.from_numpy(iq), bits, nb, cfg, [0, 1, 2, 3], calls) == (0, [])
    assert bench.steady_state_check(torch.from_numpy(iq), bits, nb, cfg, [0, 1, 2, 3], calls - 1)[0] > 0
    bits[2, 3] ^= 1
    assert bench.steady_state_check(torch.from_numpy(iq), bits, nb, cfg, [0, 1, 2, 3], calls) == (1, [2])


# ---- the output gather of a sharded call, gloo ----
def _og_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = bench.shard_streams(2 * SG_STREAMS, rank, world)
        bits, nb = _sg_demod(_sg_synth(lo, hi - lo))
        rec, gathered = bench.gather_outputs(bits, nb, world, rank, torch.device("cpu"), host_collectives=True)
        q.put((rank, rec, None if gathered is None else (gathered[0].numpy(), gathered[1].numpy())))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_output_gather_matches_single_process():
    """bench.gather_outputs (the N > 1 sub-records' output path): rank 0 holds
    every rank's rows in rank order, equal to one process demodulating the
    whole batch, and the per-rank checksums agree."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_og_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=180) for _ in range(2)], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    rec0, (bits, nb) = res[0][1], res[0][2]
    assert res[1][2] is None
    for rec in (rec0, res[1][1]):
        assert rec["gathered_rows_match_rank_checksums"] is True
        assert rec["rows"] == 2 * SG_STREAMS and rec["gather_ms"] >= 0
    rb, rnb = _sg_demod(_sg_synth(0, 2 * SG_STREAMS))
    assert np.array_equal(nb, rnb.numpy())
    assert bench.compare_rows(bits, nb, rb.numpy(), rnb.numpy())[0] == []
