#!/usr/bin/env python3
"""bench.py -- device-resident CRC throughput for the leveldb-rust block/record checksum path.

Metric (BASELINE.json): GiB/s of CRC32C over device-resident 4 KiB blocks, and the fraction of HBM3E read
bandwidth. A "step" is one batched checksum pass over one 64K x 4 KiB batch (256 MiB, BASELINE.json
configs[1]) already resident in HBM; four such batches rotate so every step reads from HBM rather than the
256 MiB Infinity Cache. N>1: one process per GPU (torch.distributed.run), each rank checksums its own
independent batches (no collective on the data path); `value` = all ranks' bytes / max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config fixed|mixed|wal] [--mode c|ref]

Steps are submitted round-robin to --streams engines (default 2: two contexts, each with its own HIP
stream and workspace), the way a storage server keeps more than one verify batch in flight: batch i+1's
workgroups start on the CUs that batch i's tail has already left. Every step is a complete, independent
launch over its own batch; nothing is skipped or cached.

Prints ONE JSON line on rank 0. `roofline.achieved` = payload bytes per launch / average duration of the
SAME launch run alone: a second timed phase launches it back to back on ONE stream, bracketed by HIP
events on that stream (this is the figure the rocprofv3 kernel trace in profiles/ must agree with, taken
with --streams 1). `traffic` comes from the rocprofv3 PMC summary in profiles/ when one exists for this
workload (tools/profile_round.sh), else null. `cpu_baseline` times the oracle's restatement of the
reference's CPU CRC on this host (rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__ as entry  # noqa: E402

METRIC = "GiB/s CRC32C over device-resident 4 KiB blocks; % of HBM3E read BW"
PEAK_GBS = 8000.0  # MI355X HBM3E peak, GB/s (MI355X_MICROARCH.md chip table, spec)
NBUF = 4


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", choices=["fixed", "mixed", "wal", "table", "snappy", "seal"], default="fixed")
    p.add_argument("--mode", choices=["c", "ref"], default="c")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=1.0, help="wall seconds of the CPU baseline sample")
    p.add_argument("--extra-out", default=None, help="also write the result dict to this file")
    p.add_argument("--host-resident", action="store_true",
                   help="fixed config starting and ending in (pinned) host memory: H2D + kernel + D2H per step "
                        "(the PCIe-inclusive end-to-end rate reported in DESIGN.md, never the headline value)")
    p.add_argument("--chunk-mib", type=int, default=32, help="host-resident pipeline chunk size")
    p.add_argument("--streams", type=int, default=2, help="engines (context + HIP stream) steps rotate over")
    return p.parse_args(argv)


class Dist:
    """torch.distributed wrapper (barrier + max-over-ranks); single-process when WORLD_SIZE is unset."""

    def __init__(self, backend=None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(self.local_rank)
            dist.init_process_group(backend)
            self.dist, self.torch, self.backend = dist, torch, backend

    def barrier(self):
        if self.dist is not None:
            if self.backend == "nccl":
                self.dist.barrier(device_ids=[self.local_rank])
            else:
                self.dist.barrier()

    def max(self, x):
        if self.dist is None:
            return x
        dev = f"cuda:{self.local_rank}" if self.backend == "nccl" else "cpu"
        t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def cuda_sync():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except ImportError:
        pass


def timed_run(dist, step, steps, warmup, engines=()):
    """W untimed steps, then exactly K steps bracketed by barrier + device sync on both sides.
    Returns the max-over-ranks wall seconds."""
    for i in range(warmup):
        step(i)
    for e in engines:
        e.sync()
    cuda_sync()
    dist.barrier()
    cuda_sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    for e in engines:
        e.sync()
    cuda_sync()
    dist.barrier()
    cuda_sync()
    elapsed = time.perf_counter() - t0
    return dist.max(elapsed), None


def launch_ms(step_on, eng, reps, windows=3):
    """Average duration of one launch run alone: `reps` launches back to back on ONE engine's stream,
    bracketed by HIP events recorded on that stream; the median of `windows` such windows (the chip's
    clock under this load wanders by ~10% from one window to the next)."""
    step_on(0, eng)
    eng.sync()
    per = []
    for _ in range(windows):
        eng.timer_start()
        for i in range(reps):
            step_on(i, eng)
        per.append(eng.timer_stop() / reps)
        eng.sync()
    return float(np.median(per))


def launch_ms_graph(step_on, eng, reps, windows=3):
    """Same as launch_ms with the `reps` launches captured once into a HIP graph and the graph replayed:
    the per-launch dispatch gap of the stream path mostly disappears, so the figure is close to the
    kernel's own duration (what rocprofv3's kernel trace reports). None if the step cannot be captured."""
    step_on(0, eng)
    eng.sync()
    try:
        g = eng.graph_capture(lambda: [step_on(i, eng) for i in range(reps)])
    except RuntimeError:
        return None
    try:
        eng.graph_launch(g)
        eng.sync()
        per = []
        for _ in range(windows):
            eng.timer_start()
            eng.graph_launch(g)
            per.append(eng.timer_stop() / reps)
            eng.sync()
    finally:
        eng.graph_destroy(g)
    return float(np.median(per))


def aggregate_gibs(bytes_per_step, steps, world, elapsed_max):
    """Whole-job throughput: every rank processed bytes_per_step * steps in at most elapsed_max."""
    return bytes_per_step * steps * world / elapsed_max / 2 ** 30


# ---------------------------------------------------------------------------------------------------
# workloads: each returns (step(i) callable, payload bytes per step, config dict, host sample for the CPU
# baseline, verify(i) callable giving the device crcs of step i for the baseline cross-check)
# ---------------------------------------------------------------------------------------------------
def workload_fixed(m, synth, engs, rank, device):
    nblk, blen = 65536, 4096
    host = [synth.splitmix_bytes(synth.SEED_FIXED + rank * NBUF + i, nblk * blen) for i in range(NBUF)]
    bufs = [m.DeviceBuffer.from_host(h, device) for h in host]
    outs = [m.DeviceBuffer(nblk * 4, device) for _ in engs]

    def step_on(i, eng):
        eng.batch_uniform(bufs[i % NBUF], nblk, blen, blen, outs[engs.index(eng)])

    step_on.graphable = True

    def crcs():  # device result for batch 0 (the CPU baseline's sample)
        step_on(0, engs[0])
        engs[0].sync()
        return outs[0].download(np.uint32, nblk)

    cfg = {"workload": "64K x 4 KiB blocks, device-resident (BASELINE configs[1])", "blocks": nblk,
           "block_bytes": blen, "batches_rotated": NBUF, "layout": "back-to-back"}
    return step_on, nblk * blen, cfg, (host[0], nblk, blen), crcs


def workload_host(m, synth, engs, rank, device, chunk_mib=32):
    nblk, blen = 65536, 4096
    pinned = m.PinnedBuffer(nblk * blen)
    pinned.array[:] = synth.splitmix_bytes(synth.SEED_FIXED + rank * NBUF, nblk * blen)

    def step_on(i, eng):
        eng.batch_host_uniform(pinned, nblk, blen, blen, chunk_bytes=chunk_mib << 20)

    cfg = {"workload": "64K x 4 KiB blocks, HOST-resident pinned buffer: H2D + kernel + D2H (end-to-end)",
           "blocks": nblk, "block_bytes": blen, "chunk_mib": chunk_mib}
    return step_on, nblk * blen, cfg, None, None


def workload_mixed(m, synth, engs, rank, device):
    sizes = synth.mixed_sizes(256 << 20, seed=synth.SEED_MIXED + rank)
    offs, total = synth.sstable_layout(sizes)
    data = synth.splitmix_bytes(synth.SEED_MIXED + 1000 + rank, total)
    d = np.zeros(len(sizes), m.DESC_DTYPE)
    d["offset"], d["length"], d["expect_rel"] = offs, sizes.astype(np.uint64) + 1, m.NO_EXPECT
    bufs = [m.DeviceBuffer.from_host(data, device) for _ in range(2)]
    dd = m.DeviceBuffer.from_host(d.view(np.uint8), device)
    outs = [m.DeviceBuffer(4 * len(sizes), device) for _ in engs]
    for e in engs:
        e.reserve(total)

    def step_on(i, eng):
        eng.batch(bufs[i % 2], total, dd, len(sizes), outs[engs.index(eng)])

    step_on.graphable = True

    cfg = {"workload": "SSTable file, block sizes 256 B-64 KiB zipf(1.1) (BASELINE configs[2])",
           "blocks": int(len(sizes)), "file_bytes": int(total), "mean_block": float(sizes.mean())}
    return step_on, int((sizes.astype(np.uint64) + 1).sum()), cfg, None, None


def workload_wal(m, synth, engs, rank, device):
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
    covered = int((first["length"].astype(np.uint64) + 1).sum())

    def step_on(i, eng):  # enqueued like the other workloads; records and their count stay on the device
        k = engs.index(eng)
        eng.wal_scan_async(dev, len(data), recs[k], maxr, counts[k])

    step_on.graphable = True

    cfg = {"workload": "WAL: 32 KiB log blocks, records n~U[1,2^k), k~U[1,16] (BASELINE configs[3])",
           "file_bytes": int(len(data)), "records": int(len(first)), "bytes_counted": "sum(1+len)"}
    return step_on, covered, cfg, None, None


def workload_table(m, synth, engs, rank, device):
    """Whole-table verify scan of a 64K x 4 KiB-block SSTable: footer, index parse on
    the host, one device verify of every trailer. The trailers are sealed once by the device writer path."""
    nblk, blen = 65536, 4096
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
    # the results land in pinned host memory (lcrc_host_alloc_pinned), as a caller that scans often would
    # keep them: the 1.5 MB copy then runs at the PCIe rate instead of through a pageable staging copy
    pinned = m.PinnedBuffer((len(blocks) + 8) * m.TBLK_DTYPE.itemsize)
    out = pinned.array.view(m.TBLK_DTYPE)
    out[:] = 0
    scanners = [m.Engine(device, m.MODE_REF) for _ in engs]
    got = scanners[0].table_scan_into(dev, len(f), out)
    if got != len(blocks) or (out["status"][:got] != 0).any():
        raise RuntimeError("table bench: the sealed table does not scan clean")

    def step_on(i, eng):  # synchronous: host footer/index parse, device verify, results back on the host
        scanners[engs.index(eng)].table_scan_into(dev, len(f), out)

    step_on.keep = pinned  # the pinned buffer lives as long as the step

    cfg = {"workload": "whole-table verify scan: 64K x 4 KiB data blocks + index (crc32fast trailers)",
           "blocks": len(blocks), "file_bytes": int(len(f))}
    return step_on, int(sum(b[1] + 1 for b in blocks)), cfg, None, None


def workload_seal(m, synth, engs, rank, device):
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

    def step_on(i, eng):  # enqueued: CRCs of every block, stored little-endian in the trailers
        eng.batch_seal(dev, len(f), dd, len(blocks))

    step_on.graphable = True
    cfg = {"workload": "writer-side trailers: 64K x 4 KiB blocks of one SSTable sealed in place",
           "blocks": len(blocks), "file_bytes": int(len(f))}
    return step_on, int(sum(b[1] + 1 for b in blocks)), cfg, None, None


def workload_snappy(m, synth, engs, rank, device):
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

    def step_on(i, eng):  # synchronous: sizes back to the host once, then decode + CRC on the device
        o, off, st = outs[engs.index(eng)]
        eng.snappy_frames_into(base, dd, nfr, o, cap, off, st)

    cfg = {"workload": "Snappy frames: 64K x (1 compressed chunk -> 4 KiB), decode + masked CRC-32C per chunk",
           "frames": nfr, "frame_bytes": len(frame)}
    return step_on, cap, cfg, None, None


def load_traffic(config, mode):
    path = os.path.join(ROOT, "profiles", f"traffic_{config}_{mode}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def cpu_baseline(orc, sample, mode, seconds, device_crcs):
    """The reference's CPU CRC restated in oracle/ (snap's SSE4.2 CRC-32C path for mode c, crc32fast's
    PCLMULQDQ path for mode ref), all usable host cores, repeated passes over the same 256 MiB batch."""
    data, nblk, blen = sample
    threads = min(16, os.cpu_count() or 1)
    algo = orc.ALGO_SSE42_C if mode == "c" else orc.ALGO_PCLMUL_REF
    crcs, secs = orc.crc_uniform_mt(data, nblk, blen, blen, threads, algo)  # warm + cross-check
    match = None
    if device_crcs is not None:
        want = crcs if mode == "ref" else np.fromiter((orc.mask(int(c)) for c in crcs), np.uint32, len(crcs))
        match = bool(np.array_equal(device_crcs(), want))
    passes, total = 0, 0.0
    while total < seconds or passes < 2:
        _, s = orc.crc_uniform_mt(data, nblk, blen, blen, threads, algo)
        total += s
        passes += 1
    gib = passes * nblk * blen / 2 ** 30
    one, one_s = 0, 0.0  # the same restatement on one core (single thread and all cores)
    while one_s < min(seconds, 1.0) or one < 1:
        _, s1 = orc.crc_uniform_mt(data, nblk, blen, blen, 1, algo)
        one_s += s1
        one += 1
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": round(gib / total, 2), "unit": "GiB/s", "cores": threads, "kind": "port",
            "single_thread": round(one * nblk * blen / 2 ** 30 / one_s, 2), "cpu_model": model,
            "host_cpus": os.cpu_count(),
            "sample": f"{passes} passes over one 64K x 4 KiB batch ({gib:.1f} GiB), "
                      f"{'snap SSE4.2 crc32c' if mode == 'c' else 'crc32fast PCLMULQDQ'} restated in oracle/, "
                      f"{threads} threads",
            "cpu_seconds": round(total * threads, 1), "matches_device": match}


def main(argv=None):
    args = parse(argv)
    dist = Dist()
    rank, world = dist.rank, dist.world
    device = dist.local_rank
    m = entry.load()
    synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
    mode = m.MODE_C if args.mode == "c" else m.MODE_REF
    flags = m.FLAG_MASK if mode == m.MODE_C else 0
    engs = [m.Engine(device, mode, flags) for _ in range(max(1, args.streams))]
    if args.host_resident:
        step_on, nbytes, cfg, sample, crcs = workload_host(m, synth, engs, rank, device, args.chunk_mib)
    else:
        step_on, nbytes, cfg, sample, crcs = {"fixed": workload_fixed, "mixed": workload_mixed, "wal": workload_wal,
                                              "table": workload_table, "seal": workload_seal,
                                              "snappy": workload_snappy}[args.config](m, synth, engs, rank, device)

    def step(i):
        step_on(i, engs[i % len(engs)])

    elapsed_max, _ = timed_run(dist, step, args.steps, args.warmup, engs)
    total_bytes = nbytes * args.steps * world
    value = aggregate_gibs(nbytes, args.steps, world, elapsed_max)
    per_launch_s = launch_ms(step_on, engs[0], args.steps) / 1e3
    graph_ms = launch_ms_graph(step_on, engs[0], args.steps) if getattr(step_on, "graphable", False) else None
    kernel_s = graph_ms / 1e3 if graph_ms else per_launch_s
    achieved = nbytes / kernel_s / 1e9
    traffic = load_traffic(args.config, args.mode)
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
        "config": dict(cfg, crc="crc32c, LevelDB-masked" if mode == m.MODE_C else "crc-32/iso-hdlc (crc32fast)",
                       parallelism=f"{world} independent shard(s), no collective",
                       streams=len(engs)),
        "pct_hbm_peak": round(100.0 * (total_bytes / elapsed_max / world) / (PEAK_GBS * 1e9), 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_GBS, 4),
                     "traffic": traffic, "launch_us": round(kernel_s * 1e6, 2),
                     "stream_launch_us": round(per_launch_s * 1e6, 2),
                     "timing": ("steps launches captured in one HIP graph, replayed on the engine stream, HIP events "
                                "on that stream, median of 3 replays" if graph_ms else
                                "one stream, launches back to back, HIP events on that stream, median of 3 windows")},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and sample is not None:
        result["cpu_baseline"] = cpu_baseline(entry.load_oracle(), sample, args.mode, args.cpu_seconds, crcs)
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


if __name__ == "__main__":
    main()
