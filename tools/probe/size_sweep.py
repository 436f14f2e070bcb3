"""Times the 4 KiB fast path at several batch sizes: separates the per-launch fixed cost from the
streaming rate (t(n) = t0 + n / rate)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
MAXNB = 262144
bufs = [m.DeviceBuffer(MAXNB * 4096) for _ in range(2)]
for i, b in enumerate(bufs):
    b.upload(synth.splitmix_bytes(0x5EED0001 + i, MAXNB * 4096))
out = m.DeviceBuffer(MAXNB * 4)
eng = m.Engine(0, 1)
for nb in (16, 256, 1024, 4096, 16384, 65536, 131072, 262144):
    res = []
    iters = 200 if nb <= 16384 else 50
    for rep in range(3):
        for i in range(3):
            eng.batch_uniform(bufs[i % 2], nb, 4096, 4096, out)
        eng.timer_start()
        for i in range(iters):
            eng.batch_uniform(bufs[i % 2], nb, 4096, 4096, out)
        res.append(eng.timer_stop() / iters)
    ms = min(res)
    print(f"nblk {nb:7d} ({nb * 4096 / 2**20:7.1f} MiB): {ms * 1000:8.1f} us  {nb * 4096 / ms / 1e6:8.1f} GB/s", flush=True)
