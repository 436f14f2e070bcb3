"""Quick device-resident throughput check of the uniform 4 KiB fast path and the general path."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
NB = 65536
BUFS = 4
bufs = [m.DeviceBuffer.from_host(synth.splitmix_bytes(0x5EED0001 + i, NB * 4096)) for i in range(BUFS)]
out = m.DeviceBuffer(NB * 4)
for mode in (1, 0):
    eng = m.Engine(0, mode)
    for i in range(5):
        eng.batch_uniform(bufs[i % BUFS], NB, 4096, 4096, out)
    eng.sync()
    iters = 100
    eng.timer_start()
    for i in range(iters):
        eng.batch_uniform(bufs[i % BUFS], NB, 4096, 4096, out)
    ms = eng.timer_stop() / iters
    gb = NB * 4096 / ms / 1e6
    print(f"fast path mode={mode}: {ms*1000:.1f} us/launch  {gb:.1f} GB/s  {gb/8000*100:.1f}% of 8 TB/s  {NB*4096/(ms*1e-3)/2**30:.1f} GiB/s")
    # general path on the same bytes via descriptors
    offs = np.arange(NB, dtype=np.uint64) * 4096
    d = np.zeros(NB, m.DESC_DTYPE); d["offset"] = offs; d["length"] = 4096; d["expect_rel"] = m.NO_EXPECT
    dd = m.DeviceBuffer.from_host(d.view(np.uint8))
    eng.reserve(NB * 4096)
    for i in range(3):
        eng.batch(bufs[i % BUFS], NB * 4096, dd, NB, out)
    eng.sync()
    eng.timer_start()
    for i in range(20):
        eng.batch(bufs[i % BUFS], NB * 4096, dd, NB, out)
    ms = eng.timer_stop() / 20
    print(f"general path mode={mode}: {ms*1000:.1f} us  {NB*4096/ms/1e6:.1f} GB/s")
    eng.close()
