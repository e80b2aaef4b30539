#!/usr/bin/env python
"""bench.py -- headline benchmark of the MI355X batched QPSK demodulation chain.

Metric (BASELINE.json): complex MSa/s through the full demod chain (batched
streams), whole job over all ranks, inputs resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5]

One step = one DeModulate call (QPSKDeModulator.cs:345-425) on every stream of
the rank's batch: matched-filter FIR -> Mueller-Muller + Costas + differential
decode -> packed bits, all on the GPU.

Headline workload (`value`): C3, the largest single-GPU configuration of
BASELINE.json (4096 streams x 2^20 complex samples per GPU, sps 4, 129-tap
RRC).  Streams are independent (QPSKDeModulator.cs:20-73), so ranks shard
streams with no data-path collective ("scaling": "weak": every rank owns its
own C3-shaped batch); the only collectives are the MAX of the timed region and
the sums of the parity / BER counters after it.  The other configs run after
the headline as `sub_records` (N=1: C2, the C4 shard, C5 and C3 with the
glibc-exact Costas trig; N>1: the C4 shard shape, 4096 streams/GPU at sps 8,
plus the RCCL scatter/gather leg of SURVEY.md 8e).

stdout carries ONE compact JSON line (<= LINE_MAX_BYTES: the driver's keys,
roofline, cpu_baseline, parity counts, GPU and CPU BER, per sub-record the
same); the full record (per-launch statistics, clocks, FIR phase samples,
framer, host ring) goes to the --detail side file, named in the line.

After each config's timed region (never inside it) the timed handle itself is
checked: one call from the initial state on every stream, whose bit rows are
compared with the CPU oracle run on the host cores (glibc trig, what .NET on
Linux calls) -- the same run is the `cpu_baseline` -- over as many streams as
fit the CPU time budget, always including the last 64 rows of the batch
(row offsets past 4 GiB at C3/C5).  Rank 0 at N=1 only; at N>1 every rank
checks the first and last two streams of its shard against the portable-trig
oracle.

--gpus N without a launcher spawns `torch.distributed.run` with N ranks
before anything touches the GPU, and exits with its status.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "qpsk-modulator-demodulator_amd")
for _p in (PKG, os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

FS = 10_000_000
ALPHA = 0.4000000059604645            # (double)0.4f, testAtDataLevel.cs:18
HBM_PEAK_GBS = 8000.0                 # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TFLOPS = 157.3              # MI355X_MICROARCH.md: peak FP32 vector (spec)
# the reference rounds every product and every sum (no FMA), so a mul or an
# add -- packed or not -- is one flop per lane-op: half the FMA peak
FP32_PEAK_UNFUSED_TFLOPS = FP32_PEAK_TFLOPS / 2
METRIC = "complex MSa/s through full demod chain (batched streams); BER vs CPU ref"

CONFIGS = {
    # BASELINE.json configs[1..4]; n = 2^20 complex samples per stream
    "c2": dict(streams=256, sps=8, span=8, impaired=False, fll=False,
               name="C2: 256 streams x 2^20 complex samples, sps=8, 65-tap RRC, clean +-1ppm LOs"),
    "c3": dict(streams=4096, sps=4, span=32, impaired=False, fll=False,
               name="C3: 4096 streams x 2^20 complex samples, sps=4, 129-tap RRC, clean +-1ppm LOs"),
    "c4": dict(streams=4096, sps=8, span=8, impaired=False, fll=False,
               name="C4 shard: 4096 streams/GPU x 2^20 complex samples, sps=8, 65-tap RRC"),
    "c5": dict(streams=8192, sps=8, span=8, impaired=True, fll=True,
               name="C5: 8192 streams x 2^20, +-5 kHz CFO + 4-tap multipath + 20 dB, FLL on"),
    # C3 with the Costas loop's own trig restated exactly (CostasLoopQpsk.cs:69-70:
    # glibc sin/cos): bit-exact by construction, not by measurement
    "c3_glibc": dict(streams=4096, sps=4, span=32, impaired=False, fll=False, costas_trig=1,
                     name="C3, glibc-exact Costas sin/cos (costas_trig=1)"),
}


def shard_streams(total: int, rank: int, world: int):
    """Contiguous stream range of one rank."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def reduce_stats(elapsed: float, counters, device=None):
    """MAX of the timed region, SUM of the counters over ranks (gloo or RCCL)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return elapsed, list(counters)
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    c = torch.tensor(list(counters), dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [int(v) for v in c.tolist()]


def load_traffic(config_key: str, kernel: str = "fir"):
    """HBM bytes per launch of one kernel (fir, loop, fll) from the committed
    rocprofv3 PMC passes (profiles/pmc_<kernel>_<config>.json, written by
    tools/pmc_traffic.py), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{kernel}_{config_key}.json")
    try:
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_quota():
    """CPUs this process may use per cgroup v2 cpu.max (None = unlimited)."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# ---------------------------------------------------------------------------
# parity of the timed handle against the CPU oracle
# ---------------------------------------------------------------------------
def compare_rows(gpu_bits, gpu_nb, ref_bits, ref_nb, gpu_syms=None, gpu_ns=None, ref_syms=None,
                 ref_ns=None, sym_exact=False):
    """Per-stream comparison of packed bit rows (+ symbols when both sides
    have them; sym_exact: a symbol that is not bit-identical fails the stream).
    Returns (mismatching stream indices, max |symbol error|)."""
    import numpy as np
    bad = []
    max_err = 0.0
    for i in range(len(ref_nb)):
        nb = int(ref_nb[i])
        ok = int(gpu_nb[i]) == nb
        if ok and nb:
            full = nb // 8
            ok = np.array_equal(gpu_bits[i, :full], ref_bits[i, :full])
            if ok and nb % 8:
                m = (0xFF << (8 - nb % 8)) & 0xFF
                ok = (int(gpu_bits[i, full]) & m) == (int(ref_bits[i, full]) & m)
        if ok and gpu_syms is not None and ref_syms is not None:
            ns = int(ref_ns[i])
            ok = int(gpu_ns[i]) == ns
            if ok and ns:
                d = np.abs(gpu_syms[i, : 2 * ns].astype(np.float64) - ref_syms[i, : 2 * ns])
                max_err = max(max_err, float(np.nanmax(d)) if d.size else 0.0)
                if sym_exact:
                    ok = np.array_equal(gpu_syms[i, : 2 * ns].view(np.uint32), ref_syms[i, : 2 * ns].view(np.uint32))
        if not ok:
            bad.append(i)
    return bad, max_err


def rows_to_host(t, idx):
    """Rows idx of a device tensor as one host numpy array, copied range by
    range (no device-side gather: the C5 batch leaves no HBM for one)."""
    import numpy as np
    parts = []
    a = 0
    while a < len(idx):
        b = a
        while b + 1 < len(idx) and idx[b + 1] == idx[b] + 1:
            b += 1
        parts.append(t[idx[a]: idx[b] + 1].cpu().numpy())
        a = b + 1
    return parts[0] if len(parts) == 1 else np.concatenate(parts)


def pick_streams(S, n_cover, tail=64):
    """Stream indices the CPU leg covers: all of them when the budget allows,
    else the first n_cover - tail and the last `tail` (the rows furthest into
    the batch buffers)."""
    if n_cover >= S:
        return list(range(S))
    head = max(1, n_cover - tail)
    return list(range(head)) + list(range(S - tail, S))


BER_STREAMS = 32      # leading streams of every rank's shard that BER is counted on


def cpu_leg(iq, bits_dev, nbits_dev, syms_dev, nsyms_dev, cfg, n, budget_s, threads, single_streams=8,
            n_cover=None, costas_trig=0):
    """CPU baseline + parity at scale: the oracle (glibc trig) on the host
    cores over a time-bounded subset of the timed batch, timed, and its bit
    rows / symbols compared with the GPU's rows of the same streams.
    n_cover: a fixed stream count instead of the time budget (N > 1: every
    rank checks the first 32 and the last 64 streams of its shard).
    Also returns the oracle's own bit rows (and counts) of the leading
    min(S, BER_STREAMS) streams, for the CPU side of the BER comparison."""
    import numpy as np
    import torch
    import oracle as O
    S = iq.shape[0]
    sps, span = cfg["sps"], cfg["span"]
    kw = dict(rrc_alpha=ALPHA, rrc_span=span, trig=O.TRIG_LIBM, enable_fll=cfg["fll"])
    # single core on the first streams: the per-stream cost that sizes the rest
    ns1 = min(S, single_streams)
    host1 = iq[:ns1].cpu().numpy()
    t0 = time.perf_counter()
    O.demod_batch_packed(host1, FS, FS // sps, n_threads=1, want_bits=False, **kw)
    dt1 = time.perf_counter() - t0
    per_stream = dt1 / ns1
    eff = min(threads, cpu_quota() or threads)
    if n_cover is None:
        n_cover = max(min(S, 64 + BER_STREAMS), int(budget_s * eff / per_stream))
    idx = pick_streams(S, n_cover)
    host = rows_to_host(iq, idx)
    want_syms = syms_dev is not None
    t0 = time.perf_counter()
    rb, rnb, rsy, rns = O.demod_batch_packed(host, FS, FS // sps, n_threads=threads,
                                             want_syms=want_syms, **kw)
    dt = time.perf_counter() - t0
    del host
    gb = rows_to_host(bits_dev, idx)
    gnb = rows_to_host(nbits_dev, idx)
    gsy = rows_to_host(syms_dev, idx) if want_syms else None
    gns = rows_to_host(nsyms_dev, idx) if want_syms else None
    bad, max_err = compare_rows(gb, gnb, rb, rnb, gsy, gns, rsy, rns, sym_exact=bool(costas_trig))
    rate = len(idx) * n / dt / 1e6
    cpu = {"value": round(rate, 2), "unit": "MSa/s", "cores": threads, "kind": "port",
           "single_core": round(ns1 * n / dt1 / 1e6, 2), "cpu_model": cpu_model(),
           "host_cpus": os.cpu_count(), "cpu_quota_cpus": cpu_quota(),
           "sample": (f"{len(idx)} of {S} streams x {n} samples "
                      + ("(the whole batch)" if len(idx) == S else
                         f"(first {len(idx) - 64} + last 64)")
                      + f", one oracle demodulator per stream (glibc trig"
                      + (", FLL on" if cfg["fll"] else "") + f") on {threads} host threads, "
                      f"{dt:.2f} s wall; single_core: first {ns1} streams on 1 thread, {dt1:.2f} s")}
    if cpu["cpu_quota_cpus"] and cpu["cpu_quota_cpus"] < threads:
        cpu["note"] = (f"the box's cgroup grants {cpu['cpu_quota_cpus']:g} CPUs of quota, so "
                       f"{threads} threads run at that rate; single_core x 128 physical cores "
                       f"= {round(cpu['single_core'] * 128, 1)} MSa/s is the unthrottled all-core "
                       "estimate (an extrapolation, not a measurement)")
    parity = {"oracle": "CPU oracle, glibc trig (what .NET on Linux calls)",
              "streams": len(idx), "first_stream": idx[0], "last_stream": idx[-1],
              "mismatching_streams": len(bad), "mismatch_examples": bad[:8],
              "max_sym_err": (round(max_err, 9) if want_syms else None),
              "sym_tol": 0.0 if costas_trig else (1e-5 if not cfg["fll"] else 1e-4),
              "max_row_offset_GiB": round(idx[-1] * iq.stride(0) * 4 / 2**30, 2)}
    if not want_syms:
        parity["note"] = "bits only: no HBM left for a symbol copy of the whole batch"
    k = min(S, BER_STREAMS)
    assert idx[:k] == list(range(k))
    return cpu, parity, (rb[:k], rnb[:k])


def portable_check(iq, bits_dev, nbits_dev, syms_dev, nsyms_dev, cfg, idx, costas_trig=0):
    """Bit-exact check (bits AND symbols) of a few streams of the timed handle
    against the oracle with the GPU's own Costas trig: the portable table
    sincos (costas_trig 0) or glibc's sin/cos (costas_trig 1, the libm oracle)."""
    import numpy as np
    import torch
    import oracle as O
    host = rows_to_host(iq, idx)
    rb, rnb, rsy, rns = O.demod_batch_packed(host, FS, FS // cfg["sps"], n_threads=len(idx),
                                             want_syms=syms_dev is not None, rrc_alpha=ALPHA,
                                             rrc_span=cfg["span"],
                                             trig=O.TRIG_LIBM if costas_trig else O.TRIG_PORTABLE,
                                             enable_fll=cfg["fll"])
    gb = rows_to_host(bits_dev, idx)
    gnb = rows_to_host(nbits_dev, idx)
    bad, err = compare_rows(gb, gnb, rb, rnb)
    sym_bad = 0
    if syms_dev is not None:
        gsy = rows_to_host(syms_dev, idx)
        gns = rows_to_host(nsyms_dev, idx)
        for i in range(len(idx)):
            ns = int(rns[i])
            if int(gns[i]) != ns or not np.array_equal(gsy[i, : 2 * ns].view(np.uint32),
                                                      rsy[i, : 2 * ns].view(np.uint32)):
                sym_bad += 1
    return len(bad), sym_bad


def steady_state_check(iq, bits_dev, nbits_dev, cfg, idx, calls):
    """The timed region's own output: the bit rows of streams idx after the
    handle's `calls` consecutive calls on the same input buffer (warmup +
    timed steps), against the libm oracle fed the same call sequence.  The
    bench re-feeds one buffer, so the streams are discontinuous at every call
    and some Costas loops sit in false lock with theta growing call by call:
    the state the timed region actually runs in, which the fresh-state legs
    do not reach.  Returns (mismatching streams, first mismatches)."""
    from concurrent.futures import ThreadPoolExecutor
    import qpsk_amd as Q
    import oracle as O
    host = rows_to_host(iq, idx)
    gb = rows_to_host(bits_dev, idx)
    gnb = rows_to_host(nbits_dev, idx)

    def one(i):
        d = O.OracleDemod(FS, FS // cfg["sps"], ALPHA, cfg["span"], enable_fll=cfg["fll"],
                          trig=O.TRIG_LIBM, ring_capacity=4096)
        for _ in range(calls - 1):
            d.demodulate_ex(host[i])
        ref, _, _ = d.demodulate_ex(host[i])
        return ref == Q.unpack_bits(gb[i], int(gnb[i]))

    with ThreadPoolExecutor(max_workers=len(idx)) as ex:
        same = list(ex.map(one, range(len(idx))))
    bad = [idx[i] for i, ok in enumerate(same) if not ok]
    return len(bad), bad[:8]


def ber_after_lock(bits_dev, nbits_dev, tx_dev, n_streams, skip_bits=8000, window=2048,
                   key_bits=64, search=512):
    """Bit errors after acquisition, with windowed realignment.

    The decoded bits of a stream are cut into windows; each window's first
    `key_bits` are located in the transmitted bits near the previous window's
    offset (the differential decoder drops the first dibit and a timing-loop
    symbol slip shifts the offset by 2 bits per symbol).  Errors are counted
    in located windows; windows that cannot be located (a slip inside the key,
    or an error in it) or whose offset changes inside them (last `key_bits`
    misaligned) are reported as `lost_windows`, not as bit errors."""
    import numpy as np

    def host(t):
        t = t[:n_streams]
        return t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)
    nb, bits, tx = host(nbits_dev), host(bits_dev), host(tx_dev)
    errs = total = lost = slips = 0
    for s in range(n_streams):
        rx = np.unpackbits(bits[s])[: int(nb[s])]
        ref = np.unpackbits(tx[s])
        rxb, refb = rx.tobytes(), ref.tobytes()
        off = None
        w = skip_bits
        while w + window <= rx.size:
            key = rxb[w: w + key_bits]
            if off is None:
                i = refb.find(key, 0, min(len(refb), w + 4 * window))
            else:
                i = refb.find(key, max(0, w + off - search), min(len(refb), w + off + search + key_bits))
            if i < 0:
                lost += 1
                w += window
                continue
            if off is not None and i - w != off:
                slips += 1
            off = i - w
            m = min(window, ref.size - (w + off))
            if m <= 0:
                break
            e = int(np.count_nonzero(rx[w: w + m] != ref[w + off: w + off + m]))
            tail_ok = rxb[w + m - key_bits: w + m] == refb[w + off + m - key_bits: w + off + m]
            if not tail_ok or e > m // 8:   # offset changed inside the window: a slip, not noise
                lost += 1
            else:
                errs += e
                total += m
            w += window
    return errs, total, lost, slips


# ---------------------------------------------------------------------------
# the RCCL leg of SURVEY.md §8e
# ---------------------------------------------------------------------------
def split_gather(synth, demod_shard, S, n, world, rank, dev, host_collectives):
    """Rank 0 synthesises the whole batch and scatters the stream shards,
    every rank demodulates its shard, and rank 0 gathers the packed bit rows
    and bit counts.  `synth(first_stream, count)` returns [count, 2n] float32
    rows (stream ids are global, so a shard is the same whatever the world
    size); `demod_shard(x)` returns (bits [S, B] uint8, n_bits [S] int64).
    Returns per-phase times (max over ranks), the gathered rows on rank 0, and
    whether every scattered shard equals the one the rank synthesised itself.
    host_collectives: gloo (CPU tensors) instead of RCCL (device tensors)."""
    import torch
    import torch.distributed as dist
    cdev = torch.device("cpu") if host_collectives else dev

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    full = synth(0, world * S).to(cdev) if rank == 0 else None
    chunks = list(full.chunk(world, dim=0)) if rank == 0 else None
    shard = torch.empty((S, 2 * n), dtype=torch.float32, device=cdev)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    dist.scatter(shard, chunks, src=0)
    sync()
    t1 = time.perf_counter()
    bits, nbits = demod_shard(shard.to(dev))
    sync()
    t2 = time.perf_counter()
    b, c = bits.to(cdev), nbits.to(cdev)
    gb = [torch.empty_like(b) for _ in range(world)] if rank == 0 else None
    gc = [torch.empty_like(c) for _ in range(world)] if rank == 0 else None
    dist.gather(b, gb, dst=0)
    dist.gather(c, gc, dst=0)
    sync()
    t3 = time.perf_counter()
    lo, _ = shard_streams(world * S, rank, world)
    same = int(torch.equal(shard, synth(lo, S).to(cdev)))
    del full, chunks
    tt = torch.tensor([t1 - t0, t2 - t1, t3 - t2], dtype=torch.float64, device=cdev)
    ok = torch.tensor([same], dtype=torch.int64, device=cdev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    ts, td, tg = (float(v) for v in tt.tolist())
    rec = {"scatter_ms": round(ts * 1e3, 3), "demod_ms": round(td * 1e3, 3),
           "gather_ms": round(tg * 1e3, 3),
           "value_with_split_gather": round(world * S * n / (ts + td + tg) / 1e6, 2),
           "shards_match_local_synth": bool(ok.item())}
    gathered = (torch.cat(gb).cpu(), torch.cat(gc).cpu()) if rank == 0 else None
    return rec, gathered


def gather_outputs(bits, nbits, world, rank, dev, host_collectives):
    """The output path of SURVEY.md §8e after a sharded call: rank 0 gathers
    every rank's packed bit rows and bit counts (dist.gather: RCCL on device
    tensors, or gloo on host copies).  Each rank also contributes a checksum
    of its own rows (all_gather of 3 int64), and rank 0 checks the gathered
    blocks against them.  Returns (record with gather time, max over ranks,
    and gathered bytes; the gathered tensors on rank 0, else None)."""
    import torch
    import torch.distributed as dist
    cdev = torch.device("cpu") if host_collectives else dev

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def checksum(b, c):
        # row bytes as int64 sums weighted by position (a swapped or shifted
        # block changes it), plus the bit counts
        w = torch.arange(1, b.shape[1] + 1, dtype=torch.int64, device=b.device)
        return torch.stack([(b.to(torch.int64) * w).sum(), c.to(torch.int64).sum(),
                            torch.tensor(b.shape[0], dtype=torch.int64, device=b.device)])

    own = checksum(bits, nbits).to(cdev)
    sums = [torch.empty_like(own) for _ in range(world)]
    dist.all_gather(sums, own)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    b, c = bits.to(cdev), nbits.to(cdev)
    gb = [torch.empty_like(b) for _ in range(world)] if rank == 0 else None
    gc = [torch.empty_like(c) for _ in range(world)] if rank == 0 else None
    dist.gather(b, gb, dst=0)
    dist.gather(c, gc, dst=0)
    sync()
    t1 = time.perf_counter()
    ok = 1
    if rank == 0:
        ok = int(all(torch.equal(checksum(gb[r], gc[r]), sums[r]) for r in range(world)))
    tt = torch.tensor([t1 - t0], dtype=torch.float64, device=cdev)
    okt = torch.tensor([ok], dtype=torch.int64, device=cdev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dist.broadcast(okt, src=0)
    nbytes = world * (b.numel() * b.element_size() + c.numel() * c.element_size())
    rec = {"gather_ms": round(float(tt.item()) * 1e3, 3),
           "gathered_GiB": round(nbytes / (1 << 30), 4),
           "rows": world * b.shape[0],
           "gathered_rows_match_rank_checksums": bool(okt.item()),
           "collective": "gloo (host copies)" if host_collectives else "RCCL gather (device tensors)"}
    return rec, ((torch.cat(gb), torch.cat(gc)) if rank == 0 else None)


TSC_BITS = "11001010011101100100100110101100" + "01110100111001011010001101101001"  # testAtDataLevel.cs:20-22


def host_ring_pass(demod, iq, S, n, steps=6, warmup=2, depth=2):
    """PCIe-inclusive rate of the host-fed streaming front-end (qpsk_rx_*, the
    ModDemodOverSDR.cs:116-183 receive loop): every call uploads S x n samples
    from pinned host slots while the previous call computes.  Untimed set-up:
    the synthetic batch is copied once into each pinned slot, which later
    submits reuse in place (an SDR driver would DMA into them)."""
    import qpsk_amd as Q
    host = iq.cpu().numpy()
    ring = Q.HostRing(demod, depth)
    pending = 0

    def submit():
        nonlocal pending
        if pending == depth:
            ring.collect()
            pending -= 1
        ring.submit(None, n)
        pending += 1

    for _ in range(depth):                 # fill every slot once
        ring.next_slot()[:, : 2 * n] = host[:, : 2 * n]
        submit()
    for _ in range(warmup):
        submit()
    while pending:
        ring.collect()
        pending -= 1
    t0 = time.perf_counter()
    for _ in range(steps):
        submit()
    while pending:
        ring.collect()
        pending -= 1
    dt = time.perf_counter() - t0
    ring.close()
    return {"value": round(S * n * steps / dt / 1e6, 2), "unit": "MSa/s",
            "ms_per_call": round(dt / steps * 1e3, 3), "depth": depth, "steps": steps,
            "h2d_GBps": round(8.0 * S * n * steps / dt / 1e9, 2),
            "note": "host pinned slots -> H2D -> demod -> D2H bits, calls overlapped; not the headline value"}


def s1_host_leg(dev, steps=10, warmup=2):
    """The literal drop-in shape (INTEGRATION.md's QPSKDeModulator shim): ONE
    stream per handle, 2^20 samples at sps 8 / 65 taps from host memory through
    qpsk_demod_process(MEM_HOST), one synchronous call after another, as
    ModDemodOverSDR.cs:136 calls DeModulate.  Timed with the host clock around
    the calls (PCIe upload, FIR, symbol loop, bits back), beside the CPU
    oracle's single core on the same row; the first call's bits are checked
    against the oracle."""
    import numpy as np
    import qpsk_amd as Q
    import oracle as O
    cfg = CONFIGS["c2"]
    n = 1 << 20
    rs = FS // cfg["sps"]
    iq, _ = Q.synth_generate(1, n, FS, rs, rrc_alpha=ALPHA, rrc_span=cfg["span"], seed=0x5159534B,
                             lo_ppm=1.0, device=dev.index)
    row = iq.cpu().numpy()
    del iq
    d = Q.BatchDemodulator(1, Q.params(FS, rs, ALPHA, cfg["span"], device=dev.index, max_samples_per_call=n))
    bits, nb, _, _ = d.process(row)
    first = (bits.copy(), nb.copy())
    for _ in range(warmup - 1):
        d.process(row)
    t0 = time.perf_counter()
    for _ in range(steps):
        d.process(row)
    dt = time.perf_counter() - t0
    d.close()
    t1 = time.perf_counter()
    rb, rnb, _, _ = O.demod_batch_packed(row, FS, rs, n_threads=1, rrc_alpha=ALPHA, rrc_span=cfg["span"],
                                         trig=O.TRIG_LIBM)
    dt1 = time.perf_counter() - t1
    bad, _ = compare_rows(first[0], first[1], rb, rnb)
    return {"kind": "drop_in", "value": round(n * steps / dt / 1e6, 2), "unit": "MSa/s",
            "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps, "warmup": warmup,
            "config": {"workload": "1 stream x 2^20 samples, sps 8, 65 taps, host memory, "
                                   "qpsk_demod_process(MEM_HOST) with S = 1 (the INTEGRATION.md shim)"},
            "cpu_single_core": round(n / dt1 / 1e6, 2),
            "parity": {"libm_oracle": {"streams": 1, "mismatching": len(bad)}},
            "note": "one stream per handle: the symbol loop is one serial recurrence on one lane, so the "
                    "GPU runs it at its per-symbol latency; batch streams per handle (BatchDeModulator, "
                    "INTEGRATION.md) for the batched rates"}


def batch_host_leg(dev, steps=5, warmup=1):
    """INTEGRATION.md's BatchDeModulator on host spans: C2's 256 streams x 2^20
    samples from ordinary (pageable) host memory per synchronous call, through
    one handle (qpsk_demod_process(MEM_HOST)) and through a group of two shards
    on the same GPU (qpsk_demod_group_process), whose shards' uploads and
    computes overlap each other.  Host clock around the calls; the two paths'
    bit rows of the last call are compared with each other, row for row."""
    import numpy as np
    import qpsk_amd as Q
    cfg = CONFIGS["c2"]
    S, n = cfg["streams"], 1 << 20
    rs = FS // cfg["sps"]
    iq, _ = Q.synth_generate(S, n, FS, rs, rrc_alpha=ALPHA, rrc_span=cfg["span"], seed=0x5159534B,
                             lo_ppm=1.0, device=dev.index)
    host = iq.cpu().numpy()
    del iq
    p = Q.params(FS, rs, ALPHA, cfg["span"], device=dev.index, max_samples_per_call=n)
    rates, rows = {}, {}
    for name, make in (("one_handle", lambda: Q.BatchDemodulator(S, p)),
                       ("group_2x_same_gpu", lambda: Q.DemodGroup(S, p, [dev.index, dev.index]))):
        d = make()
        for _ in range(warmup):
            d.process(host)
        t0 = time.perf_counter()
        for _ in range(steps):
            out = d.process(host)
        dt = time.perf_counter() - t0
        rates[name] = (round(S * n * steps / dt / 1e6, 2), round(dt / steps * 1e3, 3))
        rows[name] = out[:2]
        d.close()
    a, b = rows["one_handle"], rows["group_2x_same_gpu"]
    bad = sum(1 for s in range(S) if int(a[1][s]) != int(b[1][s]) or
              not np.array_equal(a[0][s, : (int(a[1][s]) + 7) // 8], b[0][s, : (int(b[1][s]) + 7) // 8]))
    best = max(rates, key=lambda k: rates[k][0])
    return {"kind": "drop_in", "value": rates[best][0], "unit": "MSa/s", "ms_per_step": rates[best][1],
            "steps": steps, "warmup": warmup,
            "config": {"workload": f"C2 from pageable host memory: {S} streams x 2^20 samples per synchronous "
                                   f"call (BatchDeModulator); value = {best}"},
            "one_handle": rates["one_handle"][0], "group_2x_same_gpu": rates["group_2x_same_gpu"][0],
            "parity": {"group_vs_one_handle": {"streams": S, "mismatching": bad}},
            "note": "PCIe-inclusive; [MSa/s, ms per call] per path in one_handle / group_2x_same_gpu"}


def host_ring_c3_leg(dev, chunk=1 << 18, steps=2, warmup=1):
    """C3 fed from host memory through the pinned ring (qpsk_rx_*, the
    ModDemodOverSDR.cs:116-183 receive loop at batch scale): 4096 streams x
    2^20 samples per step, uploaded in chunks of `chunk` samples per stream
    (4 chunks a step), each chunk's upload overlapping the previous chunk's
    demod.  The ring has one pinned slot per chunk, filled once before the
    timed region straight from the GPU-synthesised batch (an SDR driver would
    DMA into them), so every step replays the same 2^20 samples per stream.
    PCIe-inclusive: not the headline value.  The first chunk's bits of the
    first and last stream are checked against the oracle."""
    import numpy as np
    import torch
    import qpsk_amd as Q
    import oracle as O
    cfg = CONFIGS["c3"]
    S, n = cfg["streams"], 1 << 20
    rs = FS // cfg["sps"]
    k = n // chunk
    iq, _ = Q.synth_generate(S, n, FS, rs, rrc_alpha=ALPHA, rrc_span=cfg["span"], seed=0x5159534B,
                             lo_ppm=1.0, device=dev.index)
    d = Q.BatchDemodulator(S, Q.params(FS, rs, ALPHA, cfg["span"], device=dev.index, max_samples_per_call=chunk))
    ring = Q.HostRing(d, k)
    host0 = iq[[0, S - 1], : 2 * chunk].cpu().numpy()
    for j in range(k):                     # slot j <- chunk j of every stream (D2H into pinned memory)
        slot = torch.from_numpy(ring.next_slot())
        slot[:, : 2 * chunk].copy_(iq[:, 2 * chunk * j: 2 * chunk * (j + 1)])
        ring.submit(None, chunk)
    torch.cuda.synchronize(dev)
    del iq
    torch.cuda.empty_cache()
    bits0, nb0, _ = ring.collect()        # chunk 0 from the fresh state
    check = (bits0[[0, S - 1]].copy(), nb0[[0, S - 1]].copy())
    pending = k - 1
    for _ in range(warmup * k):
        if pending == k:
            ring.collect()
            pending -= 1
        ring.submit(None, chunk)
        pending += 1
    while pending:
        ring.collect()
        pending -= 1
    t0 = time.perf_counter()
    for _ in range(steps * k):
        if pending == k:
            ring.collect()
            pending -= 1
        ring.submit(None, chunk)
        pending += 1
    while pending:
        ring.collect()
        pending -= 1
    dt = time.perf_counter() - t0
    ring.close()
    d.close()
    rb, rnb, _, _ = O.demod_batch_packed(host0, FS, rs, n_threads=2, rrc_alpha=ALPHA, rrc_span=cfg["span"],
                                         trig=O.TRIG_LIBM)
    bad, _ = compare_rows(check[0], check[1], rb, rnb)
    return {"kind": "drop_in", "value": round(S * n * steps / dt / 1e6, 2), "unit": "MSa/s",
            "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps, "warmup": warmup,
            "config": {"workload": f"C3 from host memory: {S} streams x 2^20 samples per step through the "
                                   f"pinned ring (qpsk_rx_*), {k} chunks of {chunk} samples per stream, "
                                   f"depth {k}"},
            "h2d_GBps": round(8.0 * S * n * steps / dt / 1e9, 2),
            "parity": {"libm_oracle": {"streams": 2, "mismatching": len(bad)}},
            "note": "PCIe-inclusive (8 B/sample up, bits down); not the headline value"}


def framer_pass(bits, nbits, S, stream, reps=5):
    """§8f rank 1, measured beside the headline (never inside it): the device
    TSC search + DeModulateBytes framer over the bit rows the chain just
    produced, timed with HIP events on the framer's stream."""
    import torch
    import qpsk_amd as Q
    fr = Q.DeviceFramer(S, b"\x02", b"\x03", ring_capacity=1 << 16, device=bits.device.index)
    fr.set_stream(stream.cuda_stream)
    offs = torch.zeros(S, dtype=torch.int64, device=bits.device)
    pay = torch.zeros((S, 256), dtype=torch.uint8, device=bits.device)
    npay = torch.zeros(S, dtype=torch.int64, device=bits.device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_tsc = t_push = 0.0
    frames = 0
    for r in range(reps + 1):
        ev[0].record(stream)
        Q.tsc_find_device(bits, nbits, TSC_BITS, offs, stream.cuda_stream)
        ev[1].record(stream)
        fr.push(bits, nbits, pay, npay, None)
        ev[2].record(stream)
        stream.synchronize()
        if r:                                  # first pass allocates the hunt scratch
            t_tsc += ev[0].elapsed_time(ev[1])
            t_push += ev[1].elapsed_time(ev[2])
            frames += int((npay > 0).sum().item())
    row_bytes = float(nbits.sum().item()) / 8
    del fr
    return {"tsc_ms": round(t_tsc / reps, 4), "framer_ms": round(t_push / reps, 4),
            "frames_per_call": round(frames / reps, 1),
            "frames_per_s": round(frames / (t_push * 1e-3), 1) if t_push > 0 else None,
            "bits_GBps": round(row_bytes / (t_push / reps * 1e-3) / 1e9, 1) if t_push > 0 else None}


TIMING_SOURCE = ("in-kernel launch timestamps over the timed region: each launch's first workgroup "
                 "start to last workgroup end on the device's 100 MHz wall clock (s_memrealtime), "
                 "the span a kernel trace reports, on whichever stream the kernel ran")


def launch_stats(col):
    """Per-kernel launch statistics of one column of launch_times() (ms);
    slow_launches = launches longer than 1.3x the median (a lost dispatch
    race, a co-scheduling swing)."""
    import numpy as np
    v = np.asarray(col, dtype=np.float64)
    v = v[v > 0]
    if not v.size:
        return None
    med = float(np.median(v))
    return {"launches": int(v.size), "ms_mean": round(float(v.mean()), 4), "ms_median": round(med, 4),
            "ms_min": round(float(v.min()), 4), "ms_max": round(float(v.max()), 4),
            "ms_std": round(float(v.std()), 4), "slow_launches": int((v > 1.3 * med).sum())}


def rooflines(st, S, n, cfg, lt=None, kclk=None):
    """Per-kernel rooflines of the timed region (algorithmic
    bytes / flops per unit ÷ the kernel's mean launch time from the in-kernel
    timestamps).  lt: launch_times() rows of the timed calls; kclk:
    kernel_clocks() rows (the shader clock each kernel ran at, GHz)."""
    sps, T = cfg["sps"], cfg["span"] * cfg["sps"] + 1
    out = {}
    col = {"fll": 0, "fir": 1, "loop": 2}
    stats = {k: (launch_stats(lt[:, i]) if lt is not None and len(lt) else None) for k, i in col.items()}

    def clock(k):
        if kclk is None or not len(kclk):
            return None
        v = sorted(float(x) for x in kclk[:, col[k]] if x > 0)
        return (v[len(v) // 2], v[0], v[-1]) if v else None

    def add_clock(k, extra):
        c = clock(k)
        if c and k in out:
            out[k]["clock_ghz_median"] = round(c[0], 3)
            out[k]["clock_ghz_range"] = [round(c[1], 3), round(c[2], 3)]
            out[k].update(extra(c[0]))
            out[k]["clock_source"] = ("s_memtime / s_memrealtime over sampled wave lifetimes of every "
                                      "timed launch (qpsk_demod_kernel_clocks)")
    if st["fir"] > 0:
        fir_s = st["fir"] / 1e3
        gbs = 16.0 * S * n / fir_s / 1e9             # 8 B in + 8 B out per complex sample
        tfl = 4.0 * T * S * n / fir_s / 1e12         # real taps x complex data: 2 mul + 2 add per tap
        out["fir"] = {"kernel": "fir_tile_kernel (RRC matched filter)", "ms": round(st["fir"], 4),
                      "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(gbs / HBM_PEAK_GBS, 4),
                      "valu_tflops": round(tfl, 2), "valu_peak_tflops": FP32_PEAK_TFLOPS,
                      "valu_frac": round(tfl / FP32_PEAK_TFLOPS, 4),
                      "valu_peak_unfused_tflops": FP32_PEAK_UNFUSED_TFLOPS,
                      "valu_frac_unfused": round(tfl / FP32_PEAK_UNFUSED_TFLOPS, 4),
                      "per_unit": f"16 B and {4 * T} flop per complex sample, {S * n} samples per launch",
                      "launch_stats": stats["fir"]}
        # the unfused VALU peak at the clock the FIR actually ran at (78.65
        # TFLOP/s is quoted at 2.4 GHz)
        add_clock("fir", lambda g: {"valu_frac_unfused_at_clock":
                                    round(tfl / (FP32_PEAK_UNFUSED_TFLOPS * g / 2.4), 4)})
    if st["loop"] > 0:
        loop_s = st["loop"] / 1e3
        b = (8.0 + 0.25 / sps) * S * n               # MF samples in + packed bits out
        syms = S * n / sps
        out["loop"] = {"kernel": "loop_kernel (M&M + Costas + decode)", "ms": round(st["loop"], 4),
                       "bound": "latency (serial per-stream recurrence)",
                       "achieved": round(b / loop_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(b / loop_s / 1e9 / HBM_PEAK_GBS, 4),
                       "ns_per_symbol_per_stream": round(loop_s / (n / sps) * 1e9, 2),
                       "per_unit": f"{8 + 0.25 / sps:.4f} B per complex sample, {S * n} samples, "
                                   f"{int(syms)} symbols per launch",
                       "launch_stats": stats["loop"]}
        # shader cycles per symbol of one stream's chain (the stamped loop
        # probe's figure of merit)
        add_clock("loop", lambda g: {"cycles_per_symbol": round(loop_s * g * 1e9 / (n / sps), 1)})
    if cfg["fll"] and st["fll"] > 0:
        fll_s = st["fll"] / 1e3
        tfl = 640.0 * S * n / fll_s / 1e12
        out["fll"] = {"kernel": "fll_sys_kernel (Band-Edge FLL)", "ms": round(st["fll"], 4),
                      "bound": "latency/VALU (serial per-stream feedback)",
                      "achieved": round(16.0 * S * n / fll_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(16.0 * S * n / fll_s / 1e9 / HBM_PEAK_GBS, 4),
                      "valu_tflops": round(tfl, 2), "valu_frac": round(tfl / FP32_PEAK_TFLOPS, 4),
                      "per_unit": "16 B and 640 flop (+ one sincos) per complex sample",
                      "launch_stats": stats["fll"]}
        # shader cycles per sample of a wave (8 streams x 8 lanes): against
        # its instruction count per sample, the wave's issue rate
        add_clock("fll", lambda g: {"cycles_per_sample": round(fll_s * g * 1e9 / n, 1)})
    for v in out.values():
        v["source"] = TIMING_SOURCE
    return out


# ---------------------------------------------------------------------------
# one configuration
# ---------------------------------------------------------------------------
def run_config(key, args, rank, world, dev, steps, warmup, headline):
    import numpy as np
    import torch
    import torch.distributed as dist
    import qpsk_amd as Q

    cfg = dict(CONFIGS[key])
    trig = cfg.get("costas_trig", args.costas_trig)
    S = args.streams or cfg["streams"]
    n = args.samples
    sps, span = cfg["sps"], cfg["span"]
    rs = FS // sps
    nccl = args.dist_backend == "nccl"
    # weak scaling: the job is world*S streams, rank r owns the contiguous
    # shard [lo, hi); every stream's payload/LO/noise seeds follow its global id
    lo, hi = shard_streams(world * S, rank, world)
    assert hi - lo == S
    synth_kw = dict(rrc_alpha=ALPHA, rrc_span=span, seed=0x5159534B, lo_ppm=1.0,
                    cfo_hz=5000.0 if cfg["impaired"] else 0.0, multipath=cfg["impaired"],
                    esn0_db=20.0 if cfg["impaired"] else None, device=dev.index)
    iq, tx = Q.synth_generate(S, n, FS, rs, first_stream=lo, **synth_kw)
    p = Q.params(FS, rs, ALPHA, span, enable_fll=cfg["fll"], device=dev.index, max_samples_per_call=n,
                 loop_variant=args.loop_variant, costas_trig=trig)
    demod = Q.BatchDemodulator(S, p)
    fresh_state = demod.get_state()   # for the parity / BER call (no second handle: C5 needs ~256 GiB)
    # a real stream (torch's legacy default is handle 0, which the C ABI reads
    # as "library-owned"); torch ops and the demod then share one order
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    demod.set_stream(stream.cuda_stream)
    ms = demod.max_symbols(n)
    bits = torch.zeros((S, ((2 * ms + 7) // 8 + 127) // 64 * 64), dtype=torch.uint8, device=dev)
    nbits = torch.zeros(S, dtype=torch.int64, device=dev)

    # pipelined calls (qpsk_demod_process_async): call k+1's front stage (FIR,
    # or FLL when on) overlaps call k's symbol loop; --serial-calls runs each
    # call's stages back to back on one stream instead
    def step():
        if args.serial_calls:
            demod.process_device(iq, n, bits, nbits)
        else:
            demod.process_device_async(iq, n, bits, nbits)

    def drain():
        if not args.serial_calls:
            demod.pipeline_wait()

    for _ in range(warmup):
        step()
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    demod.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    st = demod.stage_times()
    lt = demod.launch_times()
    kclk = demod.kernel_clocks()
    demod.enable_timing(False)

    rec = {}
    errs = total_bits = lost = slips = 0
    bad_bits = bad_syms = n_port = 0
    libm_bad = libm_streams = 0
    steady_bad = steady_n = 0
    steady_ex, steady_freq = [], []
    cerrs = ctotal = clost = cslips = ber_cpu_ok = 0
    if not args.timed_only and not args.no_parity:
        # the last timed call's rows, before anything overwrites them: the first
        # and last two streams and the four whose Costas loop runs fastest (the
        # false locks, theta growing call by call: the hardest state to track)
        fr = np.abs(demod.stream_states()["freq"])
        hot = [int(i) for i in np.argsort(-fr, kind="stable")[:4]]
        sidx = sorted(set(([0, 1, S - 2, S - 1] if S >= 4 else list(range(S))) + hot))
        steady_freq = [round(float(fr[i]), 4) for i in hot]
        steady_bad, steady_ex = steady_state_check(iq, bits, nbits, cfg, sidx, warmup + steps)
        steady_n = len(sidx)
    fir_diag = None
    if not args.timed_only:
        # untimed: where the FIR's cycles go beside the loop kernel (pipelined
        # calls, as timed) and alone (serial calls: the FIR on an idle chip),
        # per phase and by whether a loop workgroup shared the FIR's CU
        # (qpsk_demod_enable_fir_phases), plus the FIR-alone launch time
        fir_diag = {}
        demod.enable_fir_phases(True)
        demod.enable_timing(True)
        for _ in range(4):
            step()
        drain()
        torch.cuda.synchronize(dev)
        fir_diag["phases_pipelined"] = demod.fir_phases()
        demod.enable_timing(True)
        for _ in range(4):
            demod.process_device(iq, n, bits, nbits)
        torch.cuda.synchronize(dev)
        fir_diag["phases_alone"] = demod.fir_phases()
        fir_diag["alone_rooflines"] = rooflines(demod.stage_times(), S, n, cfg, demod.launch_times(),
                                                demod.kernel_clocks())
        demod.enable_timing(False)
        demod.enable_fir_phases(False)
        # untimed: one call from the initial state on every stream of the timed
        # handle (stream starts at t=0); its rows feed parity and BER
        syms = nsyms = None
        if not cfg["fll"]:   # the FLL batches leave no HBM for a symbol copy
            try:
                syms = torch.empty((S, 2 * ms), dtype=torch.float32, device=dev)
                nsyms = torch.zeros(S, dtype=torch.int64, device=dev)
            except torch.OutOfMemoryError:
                syms = nsyms = None
        demod.set_state(fresh_state)
        demod.process_device(iq, n, bits, nbits, syms_dev=syms, n_syms_dev=nsyms)
        torch.cuda.synchronize(dev)
        errs, total_bits, lost, slips = ber_after_lock(bits, nbits, tx, min(S, BER_STREAMS))
        if not args.no_parity:
            idx = [0, 1, S - 2, S - 1] if S >= 4 else list(range(S))
            bad_bits, bad_syms = portable_check(iq, bits, nbits, syms, nsyms, cfg, idx, trig)
            n_port = len(idx)
            if not args.no_cpu_baseline:
                # every rank: the libm oracle on its own shard (N = 1: as many
                # streams as the CPU budget allows; N > 1: the first 8 and last
                # 64 of the shard, on this rank's share of the host threads)
                threads = args.cpu_threads or max(1, (os.cpu_count() or 1) // world)
                cpu, par, (rb, rnb) = cpu_leg(iq, bits, nbits, syms, nsyms, cfg, n, args.cpu_seconds, threads,
                                              n_cover=None if world == 1 else min(S, 64 + BER_STREAMS),
                                              costas_trig=trig)
                libm_bad, libm_streams = par["mismatching_streams"], par["streams"]
                # the same BER count on the CPU oracle's own bit rows of the
                # same streams ("BER vs CPU ref"): equal to the GPU's iff the
                # rows are, so a nonzero clean-channel BER is the algorithm's
                cerrs, ctotal, clost, cslips = ber_after_lock(rb, rnb, tx, min(S, BER_STREAMS))
                ber_cpu_ok = 1
                if rank == 0:
                    rec["cpu_baseline"], rec["parity_vs_libm_oracle"] = cpu, par
        del syms, nsyms
    if world > 1 and S * bits.shape[1] * world <= (8 << 30):
        # the §8e output path: every rank's bit rows (the untimed call's, or
        # the last timed call's with --timed-only) and counts to rank 0
        og, gathered = gather_outputs(bits, nbits, world, rank, dev, host_collectives=not nccl)
        del gathered
        rec["output_gather"] = og
    t_max, (errs, total_bits, lost, slips, bad_bits, bad_syms, n_port, libm_bad, libm_streams,
            steady_bad, steady_n, cerrs, ctotal, clost, cslips, ber_cpu_ok) = reduce_stats(
        elapsed, [errs, total_bits, lost, slips, bad_bits, bad_syms, n_port, libm_bad, libm_streams,
                  steady_bad, steady_n, cerrs, ctotal, clost, cslips, ber_cpu_ok],
        device=dev if nccl else None)
    if world > 1 and "parity_vs_libm_oracle" in rec:
        par = rec["parity_vs_libm_oracle"]
        par["rank0"] = {k: par.pop(k) for k in ("first_stream", "last_stream", "mismatch_examples",
                                                  "max_row_offset_GiB") if k in par}
        par["streams"] = libm_streams
        par["mismatching_streams"] = libm_bad
        par["scope"] = (f"every rank: the first 8 and the last 64 streams of its {S}-stream shard, "
                        f"summed over {world} ranks")

    value = world * S * n * steps / t_max / 1e6
    rl = rooflines(st, S, n, cfg, lt, kclk)
    if fir_diag and "fir" in rl:
        # the FIR alone (serial calls after the timed region; not `value`)
        fa = fir_diag["alone_rooflines"].get("fir")
        if fa:
            rl["fir_alone"] = dict(fa, note="serial calls after the timed region: the FIR with the chip to "
                                             "itself (untimed leg, not part of value)")
        rl["fir"]["phases"] = {"pipelined": fir_diag["phases_pipelined"], "alone": fir_diag["phases_alone"],
                               "unit": "shader cycles per sampled workgroup (every 64th), per phase",
                               "note": "shared = a symbol-loop workgroup held the FIR workgroup's CU"}
    timed = [k for k in rl if k != "fir_alone"]
    dom = max(timed, key=lambda k: rl[k]["ms"]) if timed else None
    roof = None
    if dom:
        r = rl[dom]
        roof = {"bound": r["bound"], "kernel": r["kernel"], "achieved": r["achieved"], "peak": r["peak"],
                "unit": r["unit"], "frac": r["frac"], "valu_frac": r.get("valu_frac"),
                "valu_frac_unfused": r.get("valu_frac_unfused"),
                "clock_ghz": r.get("clock_ghz_median"),
                "valu_frac_unfused_at_clock": r.get("valu_frac_unfused_at_clock"),
                "traffic": (load_traffic(key, dom) if S == cfg["streams"] and n == 1 << 20 else None)}
    rec = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "MSa/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(t_max / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32/f64",
        "data": "synthetic (GPU-generated differential QPSK, RRC, +-1ppm LO pair"
                + (", +-5kHz CFO, 4-tap multipath, 20 dB Es/N0" if cfg["impaired"] else "") + ")",
        "config": {"workload": (cfg["name"] if S == cfg["streams"] else
                                f"{cfg['name']} [run with {S} streams/GPU (--streams)]"),
                   "streams_per_gpu": S, "samples_per_stream": n,
                   "sps": sps, "taps": span * sps + 1, "fll": cfg["fll"],
                   "parallelism": f"stream-shard x{world}",
                   "costas_trig": "glibc sin/cos (bit-exact vs glibc libm)" if trig else
                                  "portable table sincos (<= 1 ulp from glibc)",
                   "calls": "serial" if args.serial_calls else
                            f"pipelined (front/back stage overlap, depth {demod.pipeline_depth()})"},
        "roofline": roof,
        "rooflines": rl,
        "stages_ms": {k: round(v, 4) for k, v in st.items()},
        "ber_after_lock": {"bit_errors": errs, "bits": total_bits,
                           "ber": (errs / total_bits) if total_bits else None,
                           "lost_windows": lost, "symbol_slips": slips,
                           "streams": min(S, BER_STREAMS) * world},
        # the same counter over the CPU oracle's rows of the same streams
        "ber_cpu": ({"bit_errors": cerrs, "bits": ctotal, "ber": (cerrs / ctotal) if ctotal else None,
                     "lost_windows": clost, "symbol_slips": cslips,
                     "equal": (cerrs, ctotal, clost, cslips) == (errs, total_bits, lost, slips)}
                    if ber_cpu_ok == world else "not measured"),
        "parity_steady_state": (
            "not checked" if (args.no_parity or args.timed_only) else
            {"streams": steady_n, "mismatching_streams": steady_bad, "calls": warmup + steps,
             "oracle": "CPU oracle, glibc trig, fed the same call sequence",
             "mismatch_examples_rank0": steady_ex,
             "fastest_costas_freq_rank0": steady_freq,
             "note": "bits of the timed region's last call after every warmup and timed call on "
                     "the one input buffer: the first and last two streams of every rank's shard and "
                     "the four with the largest |Costas freq| (false locks, rad/symbol)"}),
        "parity_vs_portable_oracle": (
            "not checked" if (args.no_parity or args.timed_only) else
            {"streams": n_port, "bit_mismatch_streams": bad_bits, "symbol_mismatch_streams": bad_syms,
             "oracle": "glibc trig (libm)" if trig else "portable trig",
             "note": "first and last two streams of every rank's shard; bits and symbols must be "
                     "bit-identical (the oracle runs the GPU's own Costas trig)"}),
        **rec,
    }
    if rec.get("cpu_baseline") is None:
        rec["cpu_baseline"] = None
    if (headline or key == "c2") and world == 1 and not args.no_framer and not args.timed_only:
        rec["framer"] = framer_pass(bits, nbits, S, stream)
    if world == 1 and not args.no_host_ring and not args.timed_only and S * n * 8 <= (4 << 30):
        rec["host_ring"] = host_ring_pass(demod, iq, S, n)
    demod.close()
    del demod, iq, tx, bits, nbits
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return rec


def split_gather_leg(args, rank, world, dev, S=256):
    """§8e scatter / demod / gather on the C2 shard shape (256 streams/rank)."""
    import torch
    import qpsk_amd as Q
    cfg = CONFIGS["c2"]
    n = args.samples
    rs = FS // cfg["sps"]
    if world * S * 2 * n * 4 > (48 << 30):
        return {"skipped": "whole batch does not fit one GPU"}
    p = Q.params(FS, rs, ALPHA, cfg["span"], device=dev.index, max_samples_per_call=n)
    demod = Q.BatchDemodulator(S, p)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    demod.set_stream(stream.cuda_stream)
    ms = demod.max_symbols(n)
    bits = torch.zeros((S, ((2 * ms + 7) // 8 + 127) // 64 * 64), dtype=torch.uint8, device=dev)
    nbits = torch.zeros(S, dtype=torch.int64, device=dev)

    def synth(first, count):
        x, _ = Q.synth_generate(count, n, FS, rs, rrc_alpha=ALPHA, rrc_span=cfg["span"],
                                seed=0x5159534B, first_stream=first, lo_ppm=1.0, device=dev.index)
        return x

    def demod_shard(x):
        demod.process_device(x, n, bits, nbits)
        return bits, nbits

    rec, _ = split_gather(synth, demod_shard, S, n, world, rank, dev,
                          host_collectives=args.dist_backend != "nccl")
    rec["streams_per_rank"] = S
    demod.close()
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    torch.cuda.empty_cache()
    return rec


# ---------------------------------------------------------------------------
# the stdout line: what the driver parses, bounded; everything else goes to
# the side file (--detail, default bench_detail.json next to bench.py)
# ---------------------------------------------------------------------------
LINE_MAX_BYTES = 12_000
HEAD_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
             "scaling", "vs_baseline", "dtype", "data", "config")
ROOF_KEYS = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "valu_frac", "clock_ghz")
CPU_KEYS = ("value", "unit", "cores", "kind", "single_core", "cpu_quota_cpus", "sample")
KERNEL_KEYS = ("ms", "achieved", "frac", "valu_frac_unfused_at_clock", "cycles_per_symbol",
               "cycles_per_sample", "clock_ghz_median")
BER_KEYS = ("ber", "bit_errors", "bits", "lost_windows", "symbol_slips", "streams", "equal")


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and d.get(k) is not None}


def _parity_counts(rec):
    """Every parity leg of one record as counts (streams checked, streams
    that differ from the oracle)."""
    out = {}
    lib = rec.get("parity_vs_libm_oracle")
    if isinstance(lib, dict):
        out["libm_oracle"] = {"streams": lib["streams"], "mismatching": lib["mismatching_streams"]}
        if lib.get("max_sym_err") is not None:
            out["libm_oracle"]["max_sym_err"] = lib["max_sym_err"]
            out["libm_oracle"]["sym_tol"] = lib["sym_tol"]
    port = rec.get("parity_vs_portable_oracle")
    if isinstance(port, dict):
        out["same_trig_oracle"] = {"streams": port["streams"], "bit_mismatching": port["bit_mismatch_streams"],
                                   "symbol_mismatching": port["symbol_mismatch_streams"]}
    st = rec.get("parity_steady_state")
    if isinstance(st, dict):
        out["steady_state"] = {"streams": st["streams"], "mismatching": st["mismatching_streams"],
                               "calls": st["calls"]}
    return out or "not checked"


def _compact_body(rec):
    body = {"roofline": _pick(rec.get("roofline"), ROOF_KEYS) or None,
            "kernels": {k: _pick(v, KERNEL_KEYS) for k, v in (rec.get("rooflines") or {}).items()},
            "stages_ms": rec.get("stages_ms"),
            "cpu_baseline": _pick(rec.get("cpu_baseline"), CPU_KEYS) or None,
            "parity": _parity_counts(rec),
            "ber": _pick(rec.get("ber_after_lock"), BER_KEYS)}
    bc = rec.get("ber_cpu")
    body["ber_cpu"] = _pick(bc, BER_KEYS) if isinstance(bc, dict) else bc
    for k in ("output_gather", "split_gather"):
        if k in rec:
            body[k] = rec[k]
    return body


def compact_record(out, detail_name):
    """The one stdout JSON line: the driver's keys, the headline's roofline,
    cpu_baseline, parity counts and BER (GPU and CPU), and per sub-record the
    same, compact.  Launch statistics, clock ranges, FIR phase samples, the
    framer and host-ring passes live in the detail file only."""
    line = {k: out[k] for k in HEAD_KEYS if k in out}
    line.update(_compact_body(out))
    subs = {}
    for key, r in (out.get("sub_records") or {}).items():
        s = {k: r[k] for k in ("value", "ms_per_step", "steps", "warmup") if k in r}
        s["workload"] = r.get("config", {}).get("workload")
        if r.get("kind") == "drop_in":
            # the drop-in's own shapes (host memory): their few fields as they are
            s.update({k: r[k] for k in ("unit", "cpu_single_core", "h2d_GBps", "one_handle", "group_2x_same_gpu",
                                        "parity", "error") if k in r})
        else:
            s.update(_compact_body(r))
        subs[key] = s
    if subs:
        line["sub_records"] = subs
    line["detail"] = detail_name
    return line


def dump_line(line):
    """Serialise the stdout line within LINE_MAX_BYTES: if it would be
    longer, the sub-records lose their per-kernel tables, then everything but
    value and ms_per_step (the detail file keeps all of it)."""
    s = json.dumps(line, separators=(",", ":"))
    for keep in (lambda k: k != "kernels", lambda k: k in ("value", "ms_per_step", "workload")):
        if len(s) <= LINE_MAX_BYTES or "sub_records" not in line:
            break
        line = dict(line, sub_records={key: {k: v for k, v in r.items() if keep(k)}
                                       for key, r in line["sub_records"].items()})
        s = json.dumps(line, separators=(",", ":"))
    # still too long (an oversized headline, or no sub-records to trim): the
    # driver would drop the whole line unparsed, so fall back to the driver's
    # keys, roofline, cpu_baseline and the detail-file name, and say so
    for keys in (HEAD_KEYS + ("roofline", "cpu_baseline", "parity", "detail"),
                 HEAD_KEYS + ("roofline", "cpu_baseline", "detail"), HEAD_KEYS + ("detail",)):
        if len(s) <= LINE_MAX_BYTES:
            break
        sys.stderr.write(f"bench.py: stdout line {len(s)} B > {LINE_MAX_BYTES} B; keeping only "
                         f"{', '.join(keys)} (the detail file has everything)\n")
        line = {k: line[k] for k in keys if k in line}
        line["truncated"] = True
        s = json.dumps(line, separators=(",", ":"))
    return s


def spawn_ranks(args):
    """--gpus N without a launcher: run N ranks under torch.distributed.run in a
    child process (this process never touches the GPU) and return its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS),
                    help="headline workload (default C3, the largest single-GPU config)")
    ap.add_argument("--sub-configs", default="auto",
                    help="comma list run after the headline as sub_records; 'auto' = c2,c4,c5,c3_glibc at N=1 "
                         "(c4: the per-GPU shard of BASELINE's 8-GPU config, the N = 1 point of its "
                         "curve), c4 at N>1; 'none' = headline only")
    ap.add_argument("--sub-steps", type=int, default=20)
    ap.add_argument("--samples", type=int, default=1 << 20)
    ap.add_argument("--loop-variant", type=int, default=0,
                    help="symbol-loop kernel shape (qpsk_demod_params.loop_variant; 0 = auto)")
    ap.add_argument("--streams", type=int, default=0, help="override streams per GPU")
    ap.add_argument("--costas-trig", type=int, default=0, choices=[0, 1],
                    help="qpsk_demod_params.costas_trig: 0 portable table sincos, 1 glibc's own sin/cos")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="default: os.cpu_count()")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU-time budget per config (x effective cores) of the oracle leg")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo + --share-gpu rehearses the N>1 path on a one-GPU box")
    ap.add_argument("--timed-only", action="store_true",
                    help="warmup + timed steps of the headline only (no parity, BER, framer, "
                         "split/gather, host ring, CPU baseline, sub-records): the command rocprofv3 "
                         "traces, so its kernel averages are the timed region's")
    ap.add_argument("--no-host-ring", action="store_true",
                    help="skip the PCIe-inclusive host-ring pass (N=1, batches <= 4 GiB: C2)")
    ap.add_argument("--no-drop-in", action="store_true",
                    help="skip the drop-in shape legs (N=1: one stream per handle from host memory, C3 "
                         "through the pinned host ring)")
    ap.add_argument("--no-framer", action="store_true",
                    help="skip the device TSC + framer pass measured beside the headline")
    ap.add_argument("--no-split-gather", action="store_true",
                    help="skip the RCCL scatter/demod/gather pass that runs when N > 1")
    ap.add_argument("--serial-calls", action="store_true",
                    help="synchronous process() per step (no front/back stage overlap)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every rank uses cuda:0 (rehearsal only; numbers meaningless)")
    ap.add_argument("--detail", default="",
                    help="side file for the full record (launch stats, clocks, FIR phases, framer, "
                         "host ring); default bench_detail.json next to bench.py")
    args = ap.parse_args()
    if args.timed_only:
        args.no_parity = args.no_framer = args.no_split_gather = True
        args.no_host_ring = args.no_cpu_baseline = args.no_drop_in = True
        args.sub_configs = "none"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))

    # the JSON line is the only thing on stdout: native libraries (gloo, HIP)
    # print to fd 1 too, so fd 1 points at stderr until the line is written
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    local = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    out = run_config(args.config, args, rank, world, dev, args.steps, args.warmup, headline=True)
    subs = args.sub_configs
    if subs == "auto":
        subs = "c2,c4,c5,c3_glibc" if world == 1 else "c4"
    sub = {}
    for key in [k for k in subs.split(",") if k and k != "none" and k != args.config]:
        r = run_config(key, args, rank, world, dev, args.sub_steps, 1, headline=False)
        for k in ("metric", "unit", "n_gpus", "higher_is_better", "scaling", "vs_baseline", "dtype"):
            r.pop(k, None)
        sub[key] = r
    if world == 1 and not args.no_drop_in:
        # the drop-in's own shapes, host memory in: one stream
        # per handle, and C3 through the pinned ring.  PCIe-inclusive, never `value`
        for key, leg in (("s1_host", s1_host_leg), ("batch_host_c2", batch_host_leg),
                         ("host_ring_c3", host_ring_c3_leg)):
            try:
                sub[key] = leg(dev)
            except Exception as e:       # a failed side leg must not cost the headline line
                sub[key] = {"kind": "drop_in", "error": f"{type(e).__name__}: {e}"[:300]}
            torch.cuda.empty_cache()
    if sub:
        out["sub_records"] = sub
    if world > 1 and not args.no_split_gather:
        out["split_gather"] = split_gather_leg(args, rank, world, dev)
    sys.stdout.flush()
    if rank == 0:
        detail = os.path.abspath(args.detail or os.path.join(ROOT, "bench_detail.json"))
        try:
            with open(detail, "w") as f:
                json.dump(out, f, indent=1)
            name = os.path.relpath(detail, ROOT) if detail.startswith(ROOT + os.sep) else detail
        except OSError as e:
            name = f"not written ({e})"
        os.write(json_fd, (dump_line(compact_record(out, name)) + "\n").encode())
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
