"""Per-launch durations of the fast path over a long back-to-back run (one stream, HIP events carried by every
launch): does one k_windows<true> launch slow down after some milliseconds of sustained HBM load?
Prints the median launch time of each stretch of 50 launches. Usage: long_run.py [LAUNCHES]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
NB = 65536
K = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
bufs = [m.DeviceBuffer.from_host(synth.splitmix_bytes(0x5EED0001 + i, NB * 4096), 0) for i in range(4)]
outs = [m.DeviceBuffer(NB * 4, 0) for _ in range(2)]
engs = [m.Engine(0, m.MODE_C, m.FLAG_MASK) for _ in range(2)]
for i in range(8):
    engs[i % 2].batch_uniform(bufs[i % 4], NB, 4096, 4096, outs[i % 2])
for e in engs:
    e.sync()
time.sleep(0.5)
# stretches of 50 launches, each timed by the events its first and last launches carry (two streams alternating)
res = []
t0 = time.perf_counter()
for s in range(K // 50):
    engs[0].timer_kernels(0)
    for i in range(50):
        k = i % 2
        if i >= 48:
            engs[k].timer_kernels(1)
        engs[k].batch_uniform(bufs[i % 4], NB, 4096, 4096, outs[k])
    ms = max(engs[0].timer_span(engs[k]) for k in (0, 1))
    for e in engs:
        e.timer_kernels(2)
    res.append(ms * 1e3 / 50)
wall = time.perf_counter() - t0
for s, us in enumerate(res):
    print(f"launches {50 * s:5d}-{50 * s + 49:5d}: {us:6.2f} us a launch ({NB * 4096 / us / 1e3:7.1f} GB/s)")
print(f"wall {wall * 1e3:.1f} ms for {K} launches")
