"""Where the driver bench's wall time goes beyond the kernels: 20 steps of the fixed config as 4 queued launches
(Q = 5), timed on the host (perf_counter) from the first submission to (a) the engine's stream synchronize,
(b) a busy poll of hipStreamQuery, after a host-side idle gap of 0 .. 10 ms, against the launches' own events (first start to last end)."""
import ctypes
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
hip = ctypes.CDLL("libamdhip64.so")
hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
nb, NB, Q = 65536, 8, 5
bufs = [m.DeviceBuffer(nb * 4096) for _ in range(NB)]
for i, b in enumerate(bufs):
    b.upload(synth.splitmix_bytes(0x5EED0001 + i, nb * 4096))
outs = [m.DeviceBuffer(nb * 4) for _ in range(NB)]
eng = m.Engine(0, 1)
st = eng.stream
jobs = [m.ujobs([(bufs[(k * Q + i) % NB], nb, outs[(k * Q + i) % NB]) for i in range(Q)]) for k in range(4)]


def run(mode, idle=0.0):
    for k in range(2):
        eng.batch_uniform_queue(jobs[k], 4096, 4096)
    eng.sync()
    if idle:
        time.sleep(idle)
    t0 = time.perf_counter()
    for k in range(4):
        if k == 0:
            eng.timer_kernels(0)
        if k == 3:
            eng.timer_kernels(1)
        eng.batch_uniform_queue(jobs[k], 4096, 4096)
    t1 = time.perf_counter()
    if mode == "sync":
        eng.sync()
    else:
        while hip.hipStreamQuery(st) != 0:
            pass
        eng.sync()
    t2 = time.perf_counter()
    gpu = eng.timer_stop() * 1e3
    return (t1 - t0) * 1e6, (t2 - t0) * 1e6, gpu


for rnd in range(2):
    for mode, idle in (("sync", 0), ("spin", 0), ("sync", 1e-4), ("sync", 1e-3), ("sync", 1e-2)):
        r = np.array([run(mode, idle) for _ in range(30)])
        med = np.median(r, axis=0)
        print(f"{mode} idle {idle * 1e6:6.0f} us: submit {med[0]:.1f} us, wall {med[1]:.1f} us, gpu span {med[2]:.1f} us, "
              f"wall - gpu {med[1] - med[2]:.1f} us (p10 {np.percentile(r[:, 1] - r[:, 2], 10):.1f}, "
              f"p90 {np.percentile(r[:, 1] - r[:, 2], 90):.1f})")
