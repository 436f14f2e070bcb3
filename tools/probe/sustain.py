"""Sustained-rate probe: the fixed config run for many steps, timed per bucket of 20 steps (host clock around a
device sync), for the one-launch-per-step submission over 2 streams, the queued submission, and a torch
int32 sum over the same buffers as a memory-bound control. Shows whether the rate drops over time and whether
the drop is the kernel's or the chip's.   python tools/probe/sustain.py [BUCKETS]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as ge  # noqa: E402

m = ge.load()
synth = ge.load_synth() if hasattr(ge, "load_synth") else None
NB, BL, NBUF, BUCKET = 65536, 4096, 4, 20
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 30
rng = np.random.default_rng(1)
host = [rng.integers(0, 256, NB * BL, dtype=np.uint8) for _ in range(NBUF)]
bufs = [m.DeviceBuffer.from_host(h, 0) for h in host]
engs = [m.Engine(0, m.MODE_C, m.FLAG_MASK) for _ in range(2)]
outs = [[m.DeviceBuffer(NB * 4, 0) for _ in range(NBUF)] for _ in engs]
tb = [torch.from_numpy(h).cuda().view(torch.int32) for h in host]


def s2(i):
    k = i % 2
    engs[k].batch_uniform(bufs[i % NBUF], NB, BL, BL, outs[k][i % NBUF])


qj = [m.ujobs([(bufs[(i + j) % NBUF], NB, outs[0][(i + j) % NBUF]) for j in range(5)]) for i in range(NBUF)]


def q5(i):
    if i % 5 == 0:
        engs[0].batch_uniform_queue(qj[(i // 5) % NBUF], BL, BL)


acc = torch.zeros((), dtype=torch.int64, device="cuda")


def tsum(i):
    acc.add_(tb[i % NBUF].sum())


def sync():
    for e in engs:
        e.sync()
    torch.cuda.synchronize()


for name, f in (("s2", s2), ("q5", q5), ("torch_sum", tsum), ("s2_again", s2)):
    for i in range(10):
        f(i)
    sync()
    rates = []
    for b in range(nb):
        t0 = time.perf_counter()
        for i in range(BUCKET):
            f(b * BUCKET + i)
        sync()
        dt = time.perf_counter() - t0
        rates.append(NB * BL * BUCKET / dt / 2 ** 30)
    print(name, "GiB/s per bucket of 20 steps:", " ".join(f"{r:.0f}" for r in rates), flush=True)
    time.sleep(2)
