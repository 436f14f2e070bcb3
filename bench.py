#!/usr/bin/env python3
"""bench.py -- device-resident CRC throughput for the leveldb-rust block/record checksum path.

Metric (BASELINE.json): GiB/s of CRC32C over device-resident 4 KiB blocks, and the fraction of HBM3E read
bandwidth. A "step" is one batched checksum pass over one 64K x 4 KiB batch (256 MiB, BASELINE.json
configs[1]) already resident in HBM; four such batches rotate so every step reads from HBM rather than the
256 MiB Infinity Cache.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config fixed|mixed|wal|table|seal|snappy]
                    [--mode c|ref] [--queue Q] [--streams S]

Submission (fixed config). By default every step is one lcrc_batch_uniform launch, the launches rotated over
two engines (context + HIP stream): the fast-path kernel leaves LDS for a second workgroup per CU, so the next
step's workgroups fill each CU as soon as this step's tail leaves it (no end-of-launch spread, no launch gap).
`--queue Q` (Q > 1) hands Q steps at a time to lcrc_batch_uniform_queue instead, the way a storage server
hands over its pending verify batches: up to 32 complete batches (own buffer, own CRC output) per launch of
the queued kernel on one stream (measured at the driver's 20 steps: 5,800-5,960 GiB/s against 6,070-6,280
for the default; sustained over thousands of steps both settle at ~6,100, tools/probe/sustain.py).

N GPUs (BASELINE configs[4]): one process per GPU. Under torch.distributed.run the ranks come from the
environment; `python bench.py --gpus N` without it spawns the N rank processes itself (before anything
touches a GPU). Each rank checksums its own independent batches on device LOCAL_RANK; there is no
collective on the data path -- gloo carries only the barrier, the max-over-ranks time and the per-rank
figures. `value` = all ranks' bytes / max-over-ranks time (weak scaling).

Prints ONE JSON line on rank 0. `roofline.achieved` = algorithmic bytes per launch / average launch duration,
where the average comes from HIP events that the first and last launches of the timed region record
themselves (fixed config, both submissions; over two streams the span runs from the first launch's start to the
latest end of any stream's last launch) -- the launches rocprofv3's kernel trace reports (tools/profile_round.sh
profiles this exact command). `roofline.profile` repeats the figure from the committed rocprofv3 summary in
profiles/ for the same config. `cpu_baseline` times the oracle's restatement of the reference's CPU CRC on
this host's usable cores (rank 0, after the timed region, at any N) and cross-checks the device CRCs against it.
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__ as entry  # noqa: E402

METRIC = "GiB/s CRC32C over device-resident 4 KiB blocks; % of HBM3E read BW"
PEAK_GBS = 8000.0  # MI355X HBM3E peak, GB/s (MI355X_MICROARCH.md chip table, spec)
NBUF = 4
QMAX = 32  # batches per queued launch (MAX_QJOBS in lcrc_kernels.hip)
MIXED_QUEUE = 1  # mixed config: steps per lcrc_batch_queue submission (1: one lcrc_batch per step)
WAL_QUEUE = 1  # wal config: scans per lcrc_wal_scan_queue submission (1: one lcrc_wal_scan_async per step)
WAL_KERNELS = 4  # lcrc_wal_scan_async: header walk, record emit, window pass, range pass
TABLE_KERNELS = 4  # lcrc_table_scan_async: window pass with the index walk beside it (k_ts_windows), range pass,
# finish, decode + chunk checks + close (+ 1 with LCRC_TSCAN_SNAPPY_INDEX: the Snappy-framed index decoded first,
# k_ts_open2)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", choices=["fixed", "mixed", "wal", "table", "snappy", "seal"], default="fixed")
    p.add_argument("--timer-read-inside", action="store_true",
                   help="read the kernel-carried GPU clock before the wall clock stops (round 5's order; for A/B runs)")
    p.add_argument("--marker-timer", action="store_true",
                   help="fixed config: time the roofline with event markers after the first submission instead of "
                        "events carried by the launches")
    p.add_argument("--graph", action="store_true",
                   help="table config: replay each scanner's scan from a HIP graph (one launch per step)")
    p.add_argument("--table-sync", action="store_true",
                   help="table config: time the synchronous lcrc_table_scan (results to pinned host memory)")
    p.add_argument("--mode", choices=["c", "ref"], default="c")
    p.add_argument("--compression", type=int, choices=[0, 1], default=0,
                   help="table config: 1 = a Snappy-compressed table (the reference's default, option.rs:127) written "
                        "by the TableBuilder restatement from db_bench-style values; 0 = raw blocks")
    p.add_argument("--queue", type=int, default=None,
                   help="fixed config: 1 (default): one lcrc_batch_uniform launch per step; Q > 1: steps per "
                        "lcrc_batch_uniform_queue submission (<= 32 per launch, launches balanced); 0: all timed "
                        "steps in one queued submission. mixed config: Q > 1: steps per "
                        "lcrc_batch_queue submission on one engine; 1 (default): one lcrc_batch per step, rotated over the "
                        "engines")
    p.add_argument("--streams", type=int, default=0,
                   help="engines (context + HIP stream) the submissions rotate over (0: 1 queued, 2 per-step)")
    p.add_argument("--blocks", type=int, default=65536, help="fixed config: 4 KiB blocks per batch")
    p.add_argument("--engine", choices=["device", "host"], default="device",
                   help="host: the library's scalar host path instead of the device (device-free test of the "
                        "N-rank launcher; never a headline figure)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=1.0, help="wall seconds of the CPU baseline sample")
    p.add_argument("--extra-out", default=None, help="also write the result dict to this file")
    p.add_argument("--host-resident", action="store_true",
                   help="fixed config starting and ending in (pinned) host memory: H2D + kernel + D2H per step "
                        "(the PCIe-inclusive end-to-end rate reported in DESIGN.md, never the headline value)")
    p.add_argument("--chunk-mib", type=int, default=32, help="host-resident pipeline chunk size")
    p.add_argument("--engine-opt", action="append", default=[], metavar="NAME=V",
                   help="measurement only: an lcrc_ctx_create_ex option for every context the bench creates "
                        "(general=ranges|blocks, batch_grid_b, wal_grid_b, ts_grid, ts_blocks_div, ...); repeatable")
    p.add_argument("--assume-bus-id", default=None, help=argparse.SUPPRESS)  # test-only: --engine host's "device"
    a = p.parse_args(argv)
    a.engine_opts = {}
    for kv in a.engine_opt:
        k, _, v = kv.partition("=")
        a.engine_opts[k] = v if k == "general" else int(v)
    return a


# ---------------------------------------------------------------------------------------------------
# N ranks
# ---------------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv):
    """`bench.py --gpus N` outside torch.distributed.run: start N rank processes (RANK = LOCAL_RANK = r,
    WORLD_SIZE = N, rendezvous on 127.0.0.1) running this same command, and exit with the worst status.
    Nothing here touches a GPU: the parent only waits; rank 0 prints the line."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def bus_id_code(s):
    """A PCI bus ID "dddd:bb:dd.f" as one integer (exact in the float64 the gloo gather carries); -1 for none."""
    if not s:
        return -1
    dom, bus, df = s.split(":")
    dev, fn = df.split(".")
    return (int(dom, 16) << 16) | (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn, 16)


def bus_id_text(c):
    c = int(c)
    return None if c < 0 else f"{c >> 16:04x}:{(c >> 8) & 255:02x}:{(c >> 3) & 31:02x}.{c & 7:x}"


def check_distinct_devices(codes, shared_ok):
    """An N-rank line is the sum of N GPUs only if the ranks drive N distinct GPUs: refuse (raise) when two ranks
    resolved to one PCI bus ID, unless the test-only LCRC_RANK_DEVICE_MOD=1 put them there on purpose."""
    ids = [c for c in codes if c >= 0]
    if len(set(ids)) != len(ids) and not shared_ok:
        raise SystemExit(f"bench.py: ranks share a GPU (PCI bus IDs {[bus_id_text(c) for c in codes]}); "
                         "each rank must drive its own device (LCRC_RANK_DEVICE_MOD=1 is for tests only)")


class Dist:
    """torch.distributed over gloo (barrier, max-over-ranks, per-rank figures); single-process when
    WORLD_SIZE is unset. The data path has no collective, so no RCCL communicator is ever created."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist, self.torch = dist, torch

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, x):
        if self.dist is None:
            return x
        t = self.torch.tensor([float(x)], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, values):
        """Every rank's `values` (a list of floats), indexed by rank, on every rank."""
        if self.dist is None:
            return [list(values)]
        t = self.torch.tensor([float(v) for v in values], dtype=self.torch.float64)
        out = [self.torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.tolist() for o in out]

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def timed_run(dist, prepare, steps, warmup, engines=(), kernel_events=False, kernels_per_step=1, read_inside=False):
    """W untimed steps, then exactly K steps bracketed by barrier + device sync on both sides.
    `prepare(first, count)` returns the submissions for steps first .. first+count-1 as (submit, launches,
    steps[, engine]) tuples (argument marshalling done before the clock starts). The wall clock covers all K
    steps. The GPU clock (HIP events, no marker packet between launches, no host latency before the first kernel):
      * kernel_events, one kernel per step (the fast path): the first submission's launch records the start, every
        engine's last launch the end (lcrc_timer_kernels -> hipExtLaunchKernelGGL); the clock runs from the first
        launch's start to the latest end (lcrc_timer_span).
      * kernel_events, several dependent kernels per step: the first launch records the start; after the last
        submission the first engine's stream joins every other engine (lcrc_ctx_join) and an end event follows:
        first launch's start to the end of the last kernel of any engine.
      * otherwise: an event behind the first submission to the joined end event (steps 2..K).
    With carried events the GPU clock is read after the wall clock stops (the events are complete once the engines
    are synchronised: reading them is bookkeeping, not the steps' work); `read_inside` reads it before, as round 5.
    Returns (max-over-ranks wall seconds, this rank's wall seconds, GPU ms, launches and steps the GPU clock
    covers)."""
    mode = "marker" if not (engines and kernel_events) else "carried" if kernels_per_step == 1 else "start"

    def eng_of(sub):  # the engine a submission goes to (4th element; 0 when absent)
        return sub[3] if len(sub) > 3 else 0

    def arm(subs):
        """edge 0 before the first submission on its engine, edge 1 before each engine's last submission"""
        first = {0: eng_of(subs[0])} if subs else {}
        last = {}
        for k, sub in enumerate(subs):
            last[eng_of(sub)] = k
        return first, ({k: e for e, k in last.items()} if mode == "carried" else {})

    def submit(subs):
        first, last = arm(subs) if mode != "marker" else ({}, {})
        for k, sub in enumerate(subs):
            if k in first:
                engines[first[k]].timer_kernels(0)
            if k in last:
                engines[last[k]].timer_kernels(1)
            sub[0]()
            if mode == "marker" and k == 0 and engines and len(subs) > 1:
                engines[0].timer_start()
        return first, last

    def finish(first, last, nsubs):
        """the GPU ms of the submissions just made (waits for their end event); engines disarmed"""
        if mode == "carried":
            e0 = engines[first[0]]
            ms = max(e0.timer_span(engines[e]) for e in last.values())
            for e in engines:
                e.timer_kernels(2)
            return ms
        if not engines or (mode == "marker" and nsubs < 2):
            return None
        e0 = engines[first[0]] if first else engines[0]
        for e in engines:  # the end event closes over every engine's last kernel (lcrc_ctx_join)
            if e is not e0:
                e0.join(e)
        ms = e0.timer_stop()
        for e in engines:
            e.timer_kernels(2)
        return ms

    if warmup:
        wsubs = prepare(0, warmup)
        fw, lw = submit(wsubs)  # the warmup goes through the timed region's launch path, events included
        finish(fw, lw, len(wsubs))
    subs = prepare(warmup, steps)
    for e in engines:
        e.sync()
    dist.barrier()
    t0 = time.perf_counter()
    first, last = submit(subs)
    if mode == "carried" and not read_inside:
        for e in engines:
            e.sync()
        elapsed = time.perf_counter() - t0
        gpu_ms = finish(first, last, len(subs))
    else:  # (the end event is recorded by finish(): it must follow the last submission before the wait)
        gpu_ms = finish(first, last, len(subs))
        for e in engines:
            e.sync()
        elapsed = time.perf_counter() - t0
    dist.barrier()
    first = 1 if mode == "marker" else 0
    cov_launches = sum(sub[1] for sub in subs[first:])
    cov_steps = sum(sub[2] for sub in subs[first:])
    return dist.max(elapsed), elapsed, gpu_ms, cov_launches, cov_steps


def single_launches(w, eng, count=12):
    """Per-launch duration of ONE batch handed over alone (a reader verifying one batch): each launch carries its
    own start and end events (lcrc_timer_kernels edges 0 and 1 on the same launch) and runs with the GPU idle
    before and after it (the previous launch's end event waited for). Returns sorted durations in us."""
    us = []
    for i in range(count + 2):
        eng.timer_kernels(0)
        eng.timer_kernels(1)
        w.single(i)
        ms = eng.timer_stop()
        if i >= 2:  # the first two warm the path (code object, clocks)
            us.append(ms * 1e3)
    eng.timer_kernels(2)
    return sorted(us)


def timing_text(w, timers, one_stream):
    kps = w.cfg.get("kernels_per_step", 1)
    if w.kernel_events:
        return ("HIP events: the first timed launch's start (an event the launch carries, hipExtLaunchKernelGGL) to " +
                ("the last one's end (carried likewise)" if kps == 1 else
                 "the end of the last kernel of any stream (the streams joined, then an end event)") +
                ", / the steps (back to back, dispatch gaps included" +
                (f"; a step is {kps} dependent kernels, so this is the whole pipeline per step" if kps > 1 else "") +
                (f"; {len(timers)} streams: consecutive steps overlap, the next one's workgroups filling the CUs this "
                 "one's tail leaves, so this is the per-step rate of the stream of steps, below any single step's "
                 "duration)" if len(timers) > 1 else ")"))
    if one_stream:
        return ("HIP events on the engine stream: from the end of the timed region's first submission to its end, / the "
                "launches in between (back to back, dispatch gaps included)")
    return ("HIP events on the first engine's stream from the end of the first step to the end of the timed region "
            f"(every stream joined), / steps; with {len(timers)} streams the steps overlap, so this is wall per step of "
            "the whole pipeline, not one kernel's duration")


def aggregate_gibs(bytes_per_step, steps, world, elapsed_max):
    """Whole-job throughput: every rank processed bytes_per_step * steps in at most elapsed_max."""
    return bytes_per_step * steps * world / elapsed_max / 2 ** 30


def groups(first, count, q):
    """Split steps [first, first + count) into submissions of at most q steps, launches of <= QMAX balanced."""
    q = count if q <= 0 else q
    out = []
    i = first
    while i < first + count:
        n = min(q, first + count - i)
        out.append((i, n))
        i += n
    return out


def launches_of(n):
    return (n + QMAX - 1) // QMAX


def balanced_jobs(jobs):
    """Cut a submission into ceil(n/32) launches of near-equal size (32 + 18 would leave a short launch)."""
    k = launches_of(len(jobs))
    if k <= 1:
        return [jobs]
    per = (len(jobs) + k - 1) // k
    return [jobs[i:i + per] for i in range(0, len(jobs), per)]


class Workload:
    """run(first, count, engs): submit steps; nbytes: algorithmic bytes per step; launches(count): kernel
    launches the dominant kernel makes for `count` steps; sample / crcs: the CPU baseline's sample and the
    device's CRCs of that sample; xor(): xor of the device CRCs of step 0 (per-rank shard fingerprint)."""

    def __init__(self, run, nbytes, cfg, launches=None, sample=None, crcs=None, per_step_sync=False, engines=None,
                 kernel_events=False, kernels_per_step=1):
        self.run, self.nbytes, self.cfg = run, nbytes, cfg
        # kernel launches one step makes (the profile summary recomputes the line's measure from the kernel trace)
        self.cfg["kernels_per_step"] = kernels_per_step
        self.launches = launches or (lambda count: count)
        self.sample, self.crcs = sample, crcs
        self.per_step_sync = per_step_sync
        self.engines = engines  # the engines the steps run on, when not the bench's own
        self.kernel_events = kernel_events  # the launches can carry the roofline's events (queued fast path)
        self.single = None  # single(i): one launch of the dominant kernel (or one whole scan), alone on the GPU
        self.bound = "hbm"  # the measured limiter of the dominant kernel (roofline.bound)


# ---------------------------------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------------------------------
def workload_fixed(m, synth, engs, rank, device, args):
    nblk, blen = args.blocks, 4096
    host = [synth.splitmix_bytes(synth.SEED_FIXED + rank * NBUF + i, nblk * blen) for i in range(NBUF)]
    bufs = [m.DeviceBuffer.from_host(h, device) for h in host]
    outs = [[m.DeviceBuffer(nblk * 4, device) for _ in range(NBUF)] for _ in engs]
    q = args.queue

    if q == 1:  # one lcrc_batch_uniform launch per step, rotated over the engines
        def run(first, count):
            return [(lambda k=i % len(engs), i=i: engs[k].batch_uniform(bufs[i % NBUF], nblk, blen, blen,
                                                                        outs[k][i % NBUF]), 1, 1, i % len(engs))
                    for i in range(first, first + count)]
        run.prepares = True

        launches = lambda count: count  # noqa: E731
        sub = f"one lcrc_batch_uniform launch per step, rotated over {len(engs)} streams"
    else:
        def run(first, count):
            subs = []
            for g, (i0, n) in enumerate(groups(first, count, q)):
                k = g % len(engs)
                jobs = [(bufs[i % NBUF], nblk, outs[k][i % NBUF]) for i in range(i0, i0 + n)]
                for part in balanced_jobs(jobs):
                    arr = m.ujobs(part)
                    subs.append((lambda e=engs[k], a=arr: e.batch_uniform_queue(a, blen, blen), 1, len(part), k))
            return subs
        run.prepares = True

        launches = lambda count: sum(launches_of(n) for _, n in groups(0, count, q))  # noqa: E731
        sub = ("lcrc_batch_uniform_queue: the timed steps in one submission" if q <= 0 else
               f"lcrc_batch_uniform_queue: {q} steps per submission") + f", <= {QMAX} batches per launch"

    def crcs():  # device result for batch 0 (the CPU baseline's sample)
        engs[0].batch_uniform(bufs[0], nblk, blen, blen, outs[0][0])
        engs[0].sync()
        return outs[0][0].download(np.uint32, nblk)

    cfg = {"workload": f"{nblk // 1024}K x 4 KiB blocks, device-resident (BASELINE configs[1])", "blocks": nblk,
           "block_bytes": blen, "batches_rotated": NBUF, "layout": "back-to-back", "submission": sub}
    w = Workload(run, nblk * blen, cfg, launches, ("uniform", host[0], nblk, blen), crcs,
                 kernel_events=not args.marker_timer)
    if q == 1:  # one batch handed over alone: the launch with nothing before or after it on the GPU
        w.single = lambda i: engs[0].batch_uniform(bufs[i % NBUF], nblk, blen, blen, outs[0][i % NBUF])
    return w


def workload_fixed_host(m, synth, rank, args):
    """--engine host: the same batches through the library's scalar host path (device-free test)."""
    nblk, blen = args.blocks, 4096
    host = [synth.splitmix_bytes(synth.SEED_FIXED + rank * NBUF + i, nblk * blen) for i in range(NBUF)]
    mode = m.MODE_C if args.mode == "c" else m.MODE_REF
    last = {}

    def one(i):
        d = host[i % NBUF]
        c = np.array([m.value(d[b * blen:(b + 1) * blen], mode) for b in range(nblk)], np.uint32)
        return np.array([m.mask(int(x)) for x in c], np.uint32) if mode == m.MODE_C else c

    def run(first, count):
        for i in range(first, first + count):
            last[i % NBUF] = one(i)

    cfg = {"workload": f"{nblk} x 4 KiB blocks on the HOST scalar path (launcher test, not a GPU figure)",
           "blocks": nblk, "block_bytes": blen}
    return Workload(run, nblk * blen, cfg, None, None, lambda: one(0))


def workload_host(m, synth, engs, rank, device, args):
    nblk, blen = args.blocks, 4096
    pinned = m.PinnedBuffer(nblk * blen)
    pinned.array[:] = synth.splitmix_bytes(synth.SEED_FIXED + rank * NBUF, nblk * blen)

    def run(first, count):
        for i in range(first, first + count):
            engs[i % len(engs)].batch_host_uniform(pinned, nblk, blen, blen, chunk_bytes=args.chunk_mib << 20)

    run.keep = pinned
    cfg = {"workload": "64K x 4 KiB blocks, HOST-resident pinned buffer: H2D + kernel + D2H (end-to-end)",
           "blocks": nblk, "block_bytes": blen, "chunk_mib": args.chunk_mib}
    return Workload(run, nblk * blen, cfg, None, None, None, per_step_sync=True)


def workload_mixed(m, synth, engs, rank, device, args):
    sizes = synth.mixed_sizes(256 << 20, seed=synth.SEED_MIXED + rank)
    offs, total = synth.sstable_layout(sizes)
    data = synth.splitmix_bytes(synth.SEED_MIXED + 1000 + rank, total)
    lens = sizes.astype(np.uint64) + 1
    d = np.zeros(len(sizes), m.DESC_DTYPE)
    d["offset"], d["length"], d["expect_rel"] = offs, lens, m.NO_EXPECT
    bufs = [m.DeviceBuffer.from_host(data, device) for _ in range(2)]
    dd = m.DeviceBuffer.from_host(d.view(np.uint8), device)
    outs = [m.DeviceBuffer(4 * len(sizes), device) for _ in engs]
    for e in engs:
        e.reserve(total)

    q = args.queue
    if q == 1:  # one lcrc_batch per step, rotated over the engines
        def run(first, count):
            for i in range(first, first + count):
                k = i % len(engs)
                engs[k].batch(bufs[i % 2], total, dd, len(sizes), outs[k])
        launches = None
        sub = f"one lcrc_batch per step, rotated over {len(engs)} streams"
    else:  # lcrc_batch_queue: q steps per submission, the two passes pipelined across them (window pass of
        # step i+1 beside the range pass of step i)
        qouts = [m.DeviceBuffer(4 * len(sizes), device) for _ in range(2)]

        def run(first, count):
            subs = []
            for g, (i0, n) in enumerate(groups(first, count, q)):
                k = g % len(engs)
                arr = m.gjobs([(bufs[i % 2], total, dd, len(sizes), qouts[i % 2]) for i in range(i0, i0 + n)])
                subs.append((lambda e=engs[k], a=arr: e.batch_queue(a), n, n, k))
            return subs
        run.prepares = True
        launches = lambda count: count  # noqa: E731  (one window pass per step)
        sub = f"lcrc_batch_queue of {q} steps per submission ({len(engs)} stream(s) + the context's side stream)"

    def crcs():
        engs[0].batch(bufs[0], total, dd, len(sizes), outs[0])
        engs[0].sync()
        return outs[0].download(np.uint32, len(sizes))

    cfg = {"workload": "SSTable file, block sizes 256 B-64 KiB zipf(1.1) (BASELINE configs[2])",
           "blocks": int(len(sizes)), "file_bytes": int(total), "mean_block": float(sizes.mean()), "submission": sub}
    return Workload(run, int(lens.sum()), cfg, launches, ("ranges", data, offs, lens), crcs,
                    kernels_per_step=2, kernel_events=q == 1)


def workload_wal(m, synth, engs, rank, device, args):
    w = m.LogWriter()
    payload = synth.splitmix_bytes(synth.SEED_WAL + 1000 + rank, 1 << 20)
    for n in synth.wal_lengths(256 << 20, seed=synth.SEED_WAL + rank):
        w.add_record(payload[: min(n, len(payload))] if n <= len(payload) else np.resize(payload, n))
    data = np.frombuffer(w.contents(), np.uint8)
    dev = m.DeviceBuffer.from_host(data, device)
    maxr = len(data) // 7 + 1
    recs = [m.DeviceBuffer(maxr * m.WAL_REC_DTYPE.itemsize, device) for _ in engs]
    counts = [m.DeviceBuffer(8, device) for _ in engs]
    for e in engs:
        e.reserve(len(data))
    first = engs[0].wal_scan(dev, len(data), maxr, recs[0])
    if engs[0].mode != m.MODE_REF:
        # the writer's headers hold crc32fast values (log.rs:61-64); for a CRC-32C log re-seal every header in
        # place with this mode's raw CRC (lcrc_batch_seal, {h + 6, 1 + len, -6}) so the scan verifies clean
        d = np.zeros(len(first), m.DESC_DTYPE)
        d["offset"], d["length"], d["expect_rel"] = first["header"] + 6, first["length"] + 1, -6
        dd = m.DeviceBuffer.from_host(d.view(np.uint8), device)
        seal = m.Engine(device, engs[0].mode, 0)
        seal.batch_seal(dev, len(data), dd, len(first))
        seal.sync()
        seal.close()
        data = dev.download(np.uint8, len(data))
        first = engs[0].wal_scan(dev, len(data), maxr, recs[0])
    covered = int((first["length"].astype(np.uint64) + 1).sum())
    # structure: every record lies inside its 32 KiB block, in file order, none overlapping
    h = first["header"].astype(np.uint64)
    ends = h + 7 + first["length"].astype(np.uint64)
    if len(first) and (np.any(h[1:] < ends[:-1]) or np.any((h // 32768) != ((ends - 1) // 32768))):
        raise RuntimeError("wal bench: the device scan's records overlap or straddle a block")
    if (first["status"] != 0).any():
        raise RuntimeError("wal bench: a freshly written log has a record flagged as corrupt")

    # two copies of the log, alternated per step: 2 x 268 MB > the 256 MiB Infinity Cache, so every scan reads HBM
    devs = [dev, m.DeviceBuffer.from_host(data, device)]
    q = args.queue
    if q == 1:
        def run(first_, count):  # records and their count stay on the device
            for i in range(first_, first_ + count):
                k = i % len(engs)
                engs[k].wal_scan_async(devs[i % 2], len(data), recs[k], maxr, counts[k])
        run.keep = devs
        launches = None
        sub = f"one lcrc_wal_scan_async per step, rotated over {len(engs)} streams"
    else:  # lcrc_wal_scan_queue: q scans per submission (header walks of all first, window passes back to back)
        qrecs = [m.DeviceBuffer(maxr * m.WAL_REC_DTYPE.itemsize, device) for _ in range(q)]
        qcounts = [m.DeviceBuffer(8, device) for _ in range(q)]

        def run(first_, count):
            subs = []
            for g, (i0, n) in enumerate(groups(first_, count, q)):
                k = g % len(engs)
                arr = m.wjobs([(devs[j % 2], len(data), qrecs[j], maxr, qcounts[j]) for j in range(n)])
                subs.append((lambda e=engs[k], a=arr: e.wal_scan_queue(a), n, n, k))
            return subs
        run.prepares = True
        run.keep = devs
        launches = lambda count: count  # noqa: E731  (one window pass per step)
        sub = f"lcrc_wal_scan_queue of {q} scans per submission ({len(engs)} stream(s) + the context's side stream)"

    cfg = {"workload": "WAL: 32 KiB log blocks, records n~U[1,2^k), k~U[1,16] (BASELINE configs[3])",
           "file_bytes": int(len(data)), "records": int(len(first)), "bytes_counted": "sum(1+len)",
           "copies_rotated": 2, "submission": sub}
    sample = ("ranges_raw", data, h + 6, first["length"].astype(np.uint64) + 1)
    return Workload(run, covered, cfg, launches, sample, lambda: first["crc"].copy(), kernels_per_step=WAL_KERNELS,
                    kernel_events=q == 1)


def workload_table(m, synth, engs, rank, device, args):
    """Whole-table verify scan of a 64K x 4 KiB-block SSTable: footer, index parse on
    the device, one device verify of every trailer. The trailers are sealed once by the device writer path."""
    nblk, blen = 65536, 4096
    decoded = 0
    if args.compression:
        # every compressible data block a Snappy frame (write_block keeps it: < raw - raw/8, table.rs:489), trailers
        # sealed on the host by the writer (crc32fast over the stored bytes, table.rs:519-522)
        f, tb = synth.compressed_table(m, nblk)
        blocks = [(int(b["offset"]), int(b["size"])) for b in tb]
        dev = m.DeviceBuffer.from_host(f, device)
        for b in tb:
            if b["kind"] == m.TBLK_DATA and f[int(b["offset"] + b["size"])] == 1:
                decoded += 1
        kinds = np.asarray(tb["kind"])
        framed = f[(tb["offset"] + tb["size"]).astype(np.int64)] == 1
    else:
        f, blocks = synth.table_layout(nblk, blen, seed=synth.SEED_TABLE + rank)
        dev = m.DeviceBuffer.from_host(f, device)
        d = np.zeros(len(blocks), m.DESC_DTYPE)
        d["offset"] = [b[0] for b in blocks]
        d["length"] = [b[1] + 1 for b in blocks]
        d["expect_rel"] = [b[1] + 1 for b in blocks]
        dd = m.DeviceBuffer.from_host(d.view(np.uint8), device)
        seal = m.Engine(device, m.MODE_REF)  # the reference's trailers: crc32fast, unmasked
        seal.batch_seal(dev, len(f), dd, len(blocks))
        seal.sync()
        seal.close()
    # two copies of the table, alternated per step (2 x 269 MB > the 256 MiB Infinity Cache)
    devs = [dev, m.DeviceBuffer.from_host(dev.download(np.uint8, len(f)), device)]
    # the synchronous form's results land in pinned host memory (lcrc_host_alloc_pinned), as a caller that scans
    # often would keep them: the 1.5 MB copy then runs at the PCIe rate instead of through a pageable staging copy
    pinned = m.PinnedBuffer((len(blocks) + 8) * m.TBLK_DTYPE.itemsize)
    out = pinned.array.view(m.TBLK_DTYPE)
    out[:] = 0
    # the scanners replace the stream engines (closed first): every stream of the process takes one of its few
    # hardware queues (GPU_MAX_HW_QUEUES = 4), and two scanners whose streams share a queue run one after the other
    # (measured: 110 us per scan on two streams, as on one; 86-88 us with the scanners' streams on distinct queues)
    nscan = len(engs)
    for e in engs:
        e.close()
    scanners = [m.Engine(device, m.MODE_REF, **args.engine_opts) for _ in range(nscan)]
    got = scanners[0].table_scan_into(dev, len(f), out)
    if got != len(blocks) or (out["status"][:got] != 0).any():
        raise RuntimeError("table bench: the sealed table does not scan clean")
    # the CPU baseline's sample: every block the scan found, read_block_from_file with verify_checksum on the host
    # (the trailer CRC, and for a compressed table each frame decoded and its chunk CRCs checked); the device's
    # trailer CRCs of the same blocks are its cross-check
    scanned = out[:got].copy()
    host_file = np.asarray(f if isinstance(f, np.ndarray) else np.frombuffer(f, np.uint8))
    sample = ("table", host_file if args.compression else dev.download(np.uint8, len(f)), scanned["offset"],
              scanned["size"])
    cap = len(blocks) + 8
    res = [(m.DeviceBuffer(cap * m.TBLK_DTYPE.itemsize, device), m.DeviceBuffer(8, device), m.DeviceBuffer(8, device))
           for _ in scanners]
    dec_bytes = 0
    if args.compression:  # the decoded bytes of every frame (the decode workspace the scan reserves)
        for (off, size), fr in zip(blocks, framed):
            if fr:
                dec_bytes += len(m.snappy_frame_decode(f[off:off + size]))
    for e in scanners:
        e.table_scan_reserve(len(f), cap, dec_bytes)
    # the async form (lcrc_table_scan_async) must agree with the synchronous one before it is timed. A table written
    # with compression has a Snappy-framed index block (table.rs:430): the async scan is told so
    # (lcrc_table_scan_async_ex, LCRC_TSCAN_SNAPPY_INDEX) and decodes it on the device
    si = bool(args.compression)
    scanners[0].table_scan_async(dev, len(f), res[0][0], cap, res[0][1], res[0][2], snappy_index=si)
    scanners[0].sync()
    st = res[0][2].download(np.uint32, 2)
    n = int(res[0][1].download(np.uint64, 1)[0])
    if st[0] != 0 or n != got or res[0][0].download(m.TBLK_DTYPE, n).tobytes() != out[:got].tobytes():
        raise RuntimeError(f"table bench: the device-only scan disagrees with the synchronous scan (status {st.tolist()}, "
                           f"{n} vs {got} blocks)")

    if args.table_sync:
        def run(first, count):  # synchronous: one device scan, results back on the host
            for i in range(first, first + count):
                scanners[i % len(engs)].table_scan_into(devs[i % 2], len(f), out)
    elif args.graph:
        # each scanner's whole scan (14 launches) captured once in a HIP graph and replayed per step
        # (graph k scans copy k % 2)
        graphs = [e.graph_capture(lambda e=e, r=r, d=devs[k % 2]: e.table_scan_async(d, len(f), r[0], cap, r[1], r[2],
                                                                                     snappy_index=si))
                  for k, (e, r) in enumerate(zip(scanners, res))]

        def run(first, count):
            for i in range(first, first + count):
                k = i % len(engs)
                scanners[k].graph_launch(graphs[k])
    else:
        def run(first, count):  # device-only: enqueued, results, count and verdict stay on the device
            for i in range(first, first + count):
                k = i % len(engs)
                scanners[k].table_scan_async(devs[i % 2], len(f), res[k][0], cap, res[k][1], res[k][2], snappy_index=si)

    run.keep = (pinned, scanners, res, devs)  # (a graph holds raw pointers: the files must outlive it)
    single = None
    if not (args.table_sync or args.graph):  # one whole scan alone on the GPU (its first launch's start to its last end)
        def single(i):
            scanners[0].table_scan_async(devs[i % 2], len(f), res[0][0], cap, res[0][1], res[0][2], snappy_index=si)
    cfg = {"workload": ("whole-table verify scan: ~64K Snappy-compressed data blocks (4 KiB raw, db_bench values) + "
                        "index: block crc32fast trailers, frames decoded, every chunk's masked CRC-32C"
                        if args.compression else
                        "whole-table verify scan: 64K x 4 KiB data blocks + index (crc32fast trailers)"),
           "compression": args.compression, "decoded_bytes": int(dec_bytes), "snappy_frames": int(decoded),
           "bytes_counted": "sum(stored block + type byte): the block checksums' bytes",
           "blocks": len(blocks), "file_bytes": int(len(f)), "crc": "crc-32/iso-hdlc (crc32fast), the reference's trailers",
           "form": "lcrc_table_scan (results to pinned host)" if args.table_sync else
           "lcrc_table_scan_async captured in a HIP graph, replayed" if args.graph else "lcrc_table_scan_async",
           "snappy_index": bool(args.compression and framed[kinds == m.TBLK_INDEX].any())}
    w = Workload(run, int(sum(b[1] + 1 for b in blocks)), cfg, None, sample, lambda: scanned["crc"].copy(),
                 per_step_sync=bool(args.table_sync), engines=scanners, kernels_per_step=TABLE_KERNELS + int(si),
                 kernel_events=not (args.table_sync or args.graph))
    w.single = single
    # the compressed scan's decoders are bound by instruction issue (SQ counters: VALU + SALU per element, DESIGN.md
    # section 4), not by HBM: its fraction of 8 TB/s is reported, but the bound is not bandwidth
    w.bound = "issue" if args.compression else "hbm"
    return w


def workload_seal(m, synth, engs, rank, device, args):
    """Writer-side trailers in batch: the trailer of every block of a 64K x 4 KiB-block
    SSTable computed over content||type and stored in place (write_raw_block, table.rs:507-529, for a whole
    flush/compaction output at once); --mode ref gives the reference's crc32fast trailers."""
    nblk, blen = 65536, 4096
    f, blocks = synth.table_layout(nblk, blen, seed=synth.SEED_TABLE + rank)
    dev = m.DeviceBuffer.from_host(f, device)
    d = np.zeros(len(blocks), m.DESC_DTYPE)
    d["offset"] = [b[0] for b in blocks]
    d["length"] = [b[1] + 1 for b in blocks]
    d["expect_rel"] = [b[1] + 1 for b in blocks]
    dd = m.DeviceBuffer.from_host(d.view(np.uint8), device)
    for e in engs:
        e.reserve(len(f))
    engs[0].batch_seal(dev, len(f), dd, len(blocks))
    engs[0].sync()
    out = np.zeros(len(blocks) + 8, m.TBLK_DTYPE)
    if engs[0].table_scan_into(dev, len(f), out) != len(blocks) or (out["status"][:len(blocks)] != 0).any():
        raise RuntimeError("seal bench: the sealed table does not scan clean")

    def run(first, count):  # enqueued: CRCs of every block, stored little-endian in the trailers
        for i in range(first, first + count):
            engs[i % len(engs)].batch_seal(dev, len(f), dd, len(blocks))

    cfg = {"workload": "writer-side trailers: 64K x 4 KiB blocks of one SSTable sealed in place",
           "blocks": len(blocks), "file_bytes": int(len(f))}
    return Workload(run, int(sum(b[1] + 1 for b in blocks)), cfg, kernels_per_step=3, kernel_events=True)


def workload_snappy(m, synth, engs, rank, device, args):
    """Snappy-framed blocks: 64K frames of one compressed 4 KiB chunk each, decoded and
    every chunk's masked CRC-32C checked on the device. Bytes counted: decoded bytes."""
    nfr = 65536
    frame, raw, pos = synth.snappy_frame_synthetic(seed=synth.SEED_SNAPPY + rank)
    frame = bytearray(frame)
    frame[pos:pos + 4] = m.mask(m.crc32c_value(raw)).to_bytes(4, "little")
    blob = np.tile(np.frombuffer(bytes(frame), np.uint8), nfr)
    base = m.DeviceBuffer.from_host(blob, device)
    d = np.zeros(nfr, m.DESC_DTYPE)
    d["offset"] = np.arange(nfr, dtype=np.uint64) * len(frame)
    d["length"] = len(frame)
    d["expect_rel"] = m.NO_EXPECT
    dd = m.DeviceBuffer.from_host(d.view(np.uint8), device)
    cap = nfr * len(raw)
    outs = [(m.DeviceBuffer(cap, device), m.DeviceBuffer(8 * (nfr + 1), device), m.DeviceBuffer(nfr, device))
            for _ in engs]
    total = engs[0].snappy_frames_into(base, dd, nfr, *outs[0][:1], cap, *outs[0][1:])
    if total != cap or outs[0][2].download(np.uint8, nfr).any():
        raise RuntimeError("snappy bench: the synthetic frames do not verify")

    def run(first, count):  # synchronous: sizes back to the host once, then decode + CRC on the device
        for i in range(first, first + count):
            o, off, st = outs[i % len(engs)]
            engs[i % len(engs)].snappy_frames_into(base, dd, nfr, o, cap, off, st)

    cfg = {"workload": "Snappy frames: 64K x (1 compressed chunk -> 4 KiB), decode + masked CRC-32C per chunk",
           "frames": nfr, "frame_bytes": len(frame)}
    w = Workload(run, cap, cfg, None, None, None, per_step_sync=True)
    w.bound = "issue"  # the wave decoder: a chain of dependent elements
    return w


# ---------------------------------------------------------------------------------------------------
# evidence: committed profiles, CPU baseline
# ---------------------------------------------------------------------------------------------------
def load_traffic(config, mode):
    """The committed PMC traffic of this config (tools/summarize_profile.py): HBM bytes read + written per STEP over
    every kernel of the step (the contract's `traffic`), and the read / write split with the streaming kernel's own
    figure beside it."""
    path = os.path.join(ROOT, "profiles", f"traffic_{config}_{mode}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        t = json.load(f)
    rd, wr = t.get("step_hbm_read_bytes"), t.get("step_hbm_write_bytes")
    if rd is None or wr is None:
        return {"traffic": t.get("hbm_bytes_per_launch")}
    return {"traffic": rd + wr, "detail": {
        "step_read_bytes": round(rd), "step_write_bytes": round(wr), "stream_kernel": t.get("kernel"),
        "stream_kernel_read_bytes": round(t.get("hbm_read_bytes_per_launch", 0)),
        "stream_kernel_write_bytes": round(t.get("hbm_write_bytes_per_launch", 0)), "source": t.get("source")}}


def load_profile(config, mode, streams=2):
    """The newest committed rocprofv3 summary of this config (tools/profile_round.sh) taken with the same stream
    count (one-stream profiles carry an `s1` round tag, e.g. r03s1_*): the dominant kernel's average duration and
    the roofline fraction it implies for the bytes per launch of that run."""
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_{mode}_summary.json")))
    cands = [p for p in cands if os.path.basename(p).split("_")[0].endswith("s1") == (streams == 1)]
    for path in reversed(cands):
        with open(path) as f:
            s = json.load(f)
        if "frac" in s and "kernel" in s:
            out = {"file": os.path.relpath(path, ROOT), "kernel": s["kernel"], "avg_us": s["avg_us"],
                   "bytes_per_launch": s["bytes_per_launch"], "frac": s["frac"]}
            # the line's own measure recomputed from the profiled run's kernel trace (launches back to back;
            # over several streams they overlap, and avg_us is one launch's duration inside that overlap)
            for k in ("trace_launch_us", "frac_from_trace", "agreement"):
                if k in s:
                    out[k] = s[k]
            return out
    return None


def usable_cpus():
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota when one is set (a GPU
    box's share of a large host is a quota, not an affinity mask)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_baseline(orc, m, sample, mode, seconds, device_crcs):
    """The reference's CPU CRC restated in oracle/ (snap's SSE4.2 CRC-32C path for mode c, crc32fast's
    PCLMULQDQ path for mode ref) on every usable host core, repeated passes over the same sample, and the
    device's CRCs of that sample checked against it."""
    kind, data = sample[0], sample[1]
    threads, affinity, quota = usable_cpus()
    algo = orc.ALGO_SSE42_C if mode == "c" else orc.ALGO_PCLMUL_REF
    raw = kind in ("ranges_raw", "table")  # WAL records and table trailers carry the raw (unmasked) crc
    label = f"{'snap SSE4.2 crc32c' if mode == 'c' else 'crc32fast PCLMULQDQ'} restated in oracle/"

    if kind == "table":
        # read_block_from_file over every block (format.rs:146-213): crc32fast trailers (the reference's), Snappy
        # frames decoded and every chunk's masked CRC-32C checked (oracle/crc_oracle.c orc_table_blocks_mt)
        offs, sizes = sample[2], sample[3]

        def fn(t):
            crcs_, st_, secs_ = orc.table_blocks_mt(data, offs, sizes, t)
            if st_.any():
                raise RuntimeError("cpu baseline: the host walk finds a bad block in the table the device scanned clean")
            return crcs_, secs_
        nbytes = int(np.asarray(sizes, np.uint64).sum()) + len(offs)
        what = f"one whole-table scan ({len(offs)} blocks, {nbytes / 2 ** 20:.0f} MiB stored)"
        label = "read_block_from_file restated in oracle/ (crc32fast PCLMULQDQ trailers, Snappy frames decoded, chunk crc32c)"
    elif kind == "uniform":
        nblk, blen = sample[2], sample[3]
        fn = lambda t: orc.crc_uniform_mt(data, nblk, blen, blen, t, algo)  # noqa: E731
        nbytes = nblk * blen
        what = f"one {nblk // 1024}K x 4 KiB batch"
    else:
        offs, lens = sample[2], sample[3]
        fn = lambda t: orc.crc_ranges_mt(data, offs, lens, t, algo)  # noqa: E731
        nbytes = int(np.asarray(lens, np.uint64).sum())
        what = f"{len(offs)} ranges, {nbytes / 2 ** 20:.0f} MiB covered"
    crcs, _ = fn(threads)  # warm + cross-check
    match = None
    if device_crcs is not None:
        want = orc.mask_array(crcs) if (mode == "c" and not raw) else crcs
        match = bool(np.array_equal(device_crcs(), want))
    passes, total = 0, 0.0
    while total < seconds or passes < 2:
        _, s = fn(threads)
        total += s
        passes += 1
    gib = passes * nbytes / 2 ** 30
    one, one_s = 0, 0.0  # the same restatement on one core (single thread and all cores)
    while one_s < min(seconds, 1.0) or one < 1:
        _, s1 = fn(1)
        one_s += s1
        one += 1
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": round(gib / total, 2), "unit": "GiB/s", "cores": threads, "kind": "port",
            "single_thread": round(one * nbytes / 2 ** 30 / one_s, 2), "cpu_model": model,
            "host_cpus": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "sample": f"{passes} passes over {what} ({gib:.1f} GiB), {label}, "
                      f"{threads} threads (every usable CPU: affinity {affinity}, cgroup quota {quota})",
            "cpu_seconds": round(total * threads, 1), "matches_device": match}


# ---------------------------------------------------------------------------------------------------
def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus, argv)
    dist = Dist()
    rank, world = dist.rank, dist.world
    device = dist.local_rank
    m = entry.load()
    if os.environ.get("LCRC_RANK_DEVICE_MOD") == "1" and args.engine == "device":
        # test-only: rank r on device r % device_count, so that N device-bound ranks can share a 1-GPU box
        # (tests/test_multi_rank_gpu.py); the driver's N-GPU runs never set it (rank r = device LOCAL_RANK)
        device = dist.local_rank % max(1, m.device_count())
    # every rank's PCI bus ID, checked before any work: N ranks on fewer GPUs would report a sum that no N GPUs made
    bus_codes = [int(r[0]) for r in dist.gather([bus_id_code(m.pci_bus_id(device) if args.engine == "device"
                                                             else args.assume_bus_id)])]
    check_distinct_devices(bus_codes, os.environ.get("LCRC_RANK_DEVICE_MOD") == "1")
    synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
    mode = m.MODE_C if args.mode == "c" else m.MODE_REF
    flags = m.FLAG_MASK if mode == m.MODE_C else 0
    if args.queue is None:
        args.queue = {"mixed": MIXED_QUEUE, "wal": WAL_QUEUE}.get(args.config, 1)
    queued = args.config in ("fixed", "mixed", "wal") and not args.host_resident and args.queue != 1
    nstreams = args.streams or (1 if queued else 2)
    if args.engine == "host":
        engs = []
        w = workload_fixed_host(m, synth, rank, args)
    else:
        engs = [m.Engine(device, mode, flags, **args.engine_opts) for _ in range(max(1, nstreams))]
        if args.host_resident:
            w = workload_host(m, synth, engs, rank, device, args)
        else:
            w = {"fixed": workload_fixed, "mixed": workload_mixed, "wal": workload_wal, "table": workload_table,
                 "seal": workload_seal, "snappy": workload_snappy}[args.config](m, synth, engs, rank, device, args)

    if getattr(w.run, "prepares", False):
        prepare = w.run
    else:  # one submission per step
        per = w.launches(1)
        prepare = lambda f, c: [(lambda i=i: w.run(i, 1), per, 1) for i in range(f, f + c)]  # noqa: E731
    timers = w.engines if w.engines else engs
    # one batch handed over alone (fixed config): timed before the warmup, so that the timed region's launches are
    # the last ones of the dominant kernel in a profiled run (tools/summarize_profile.py)
    single = single_launches(w, (w.engines or engs)[0]) if (w.single is not None and (w.engines or engs)) else None
    # this rank's fingerprint (gathered over gloo with the rates below), taken before the timed region so that
    # the timed launches are the last ones of the dominant kernel in a profiled run (tools/summarize_profile.py)
    fp = int(np.bitwise_xor.reduce(w.crcs())) if w.crcs is not None else 0
    elapsed_max, elapsed, gpu_ms, cov_launches, cov_steps = timed_run(
        dist, prepare, args.steps, args.warmup, timers, kernel_events=w.kernel_events,
        kernels_per_step=w.cfg.get("kernels_per_step", 1), read_inside=args.timer_read_inside)
    value = aggregate_gibs(w.nbytes, args.steps, world, elapsed_max)
    # this rank's per-launch figure of the dominant kernel (its own HIP events; -1 when not timed on the GPU)
    launch_us = gpu_ms * 1e3 / cov_launches if (timers and gpu_ms and cov_launches) else -1.0
    bytes_per_launch = w.nbytes * cov_steps / cov_launches if cov_launches else 0
    rows = dist.gather([rank, device, elapsed, fp, launch_us])
    per_gpu = []
    for r in rows:
        row = {"rank": int(r[0]), "device": int(r[1]), "pci_bus_id": bus_id_text(bus_codes[int(r[0])]),
               "gib_s": round(w.nbytes * args.steps / r[2] / 2 ** 30, 2),
               "pct_hbm": round(100.0 * w.nbytes * args.steps / r[2] / (PEAK_GBS * 1e9), 2),
               "crc_xor": f"{int(r[3]):08x}"}
        if r[4] > 0:
            row["launch_us"] = round(r[4], 2)
            row["frac"] = round(bytes_per_launch / (r[4] * 1e-6) / 1e9 / PEAK_GBS, 4)
        per_gpu.append(row)

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 bytes, seeds in leveldb-rust_amd/synth.py)",
        "config": dict(w.cfg, crc=w.cfg.get("crc") or ("crc32c, LevelDB-masked" if mode == m.MODE_C else
                                                          "crc-32/iso-hdlc (crc32fast)"),
                       parallelism=f"{world} independent shard(s), no collective", streams=len(engs)),
        "pct_hbm_peak": round(100.0 * (w.nbytes * args.steps * world / elapsed_max / world) / (PEAK_GBS * 1e9), 2),
        "per_gpu": per_gpu,
    }
    # profiles/ tag (tablez: the compressed table)
    prof_config = args.config + ("z" if args.compression else "")
    if timers and gpu_ms:
        one_stream = len(timers) == 1 and not w.per_step_sync
        launch_s = gpu_ms / 1e3 / cov_launches
        bytes_per_launch = w.nbytes * cov_steps / cov_launches
        achieved = bytes_per_launch / launch_s / 1e9
        tr = load_traffic(prof_config, args.mode) or {}
        if tr.get("detail"):
            tr["detail"]["step_read_x"] = round(tr["detail"]["step_read_bytes"] / bytes_per_launch, 4)
            tr["detail"]["step_write_x"] = round(tr["detail"]["step_write_bytes"] / bytes_per_launch, 4)
        result["roofline"] = {
            "bound": w.bound, "achieved": round(achieved, 1), "peak": PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / PEAK_GBS, 4), "traffic": tr.get("traffic"), "traffic_detail": tr.get("detail"),
            "bytes_per_launch": int(bytes_per_launch), "launches": cov_launches, "steps_timed_on_gpu": cov_steps,
            "launch_us": round(launch_s * 1e6, 2),
            "timing": timing_text(w, timers, one_stream),
            "clock": ("marker" if not w.kernel_events else
                      "carried" if w.cfg.get("kernels_per_step", 1) == 1 else "start"),
            "profile": load_profile(prof_config, args.mode, len(engs)),
        }
        if single:
            one = single
            med = one[len(one) // 2]
            result["roofline"]["frac_single_launch"] = round(bytes_per_launch / (med * 1e-6) / 1e9 / PEAK_GBS, 4)
            result["roofline"]["single_launch"] = {
                "launch_us_median": round(med, 2), "launch_us_min": round(one[0], 2),
                "launch_us_max": round(one[-1], 2), "launches": len(one),
                "frac_best": round(bytes_per_launch / (one[0] * 1e-6) / 1e9 / PEAK_GBS, 4),
                "timing": ("one lcrc_batch_uniform launch" if w.cfg.get("kernels_per_step", 1) == 1 else
                           f"one whole scan ({w.cfg.get('kernels_per_step')} dependent launches)") +
                          " alone on the GPU (the previous one's end waited for), its own start and end events (the "
                          "first launch's start to the last one's end); median over the launches (before the warmup)"}
    else:
        result["roofline"] = None
    # the CPU baseline (north_star: "next to the reference's own CPU CRC32C timed on the same box's host cores in the
    # same run"): rank 0, after the timed region and the final barrier -- at N > 1 too, when every rank's device work
    # is done and the host cores are free -- on rank 0's own sample, cross-checked against rank 0's device CRCs
    if rank == 0 and not args.no_cpu_baseline and w.sample is not None and args.engine == "device":
        result["cpu_baseline"] = cpu_baseline(entry.load_oracle(), m, w.sample, args.mode, args.cpu_seconds, w.crcs)
        if world > 1:
            result["cpu_baseline"]["ranks_note"] = (f"timed on rank 0 after all {world} ranks' timed regions ended "
                                                    "(barrier), on rank 0's sample")
    else:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
        if args.extra_out:
            with open(args.extra_out, "w") as f:
                json.dump(result, f, indent=1)
    for e in engs:
        e.close()
    dist.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
