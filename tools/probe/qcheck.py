"""Full-size check of the queued path of a variant build (LCRC_LIB_PATH): a Q-batch queue of 64K x 4 KiB, launched
repeatedly, must give the single-batch kernel's CRCs for every batch (sizes the parity suite does not reach)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
eng = m.Engine(0, 1)
for Q, nb in ((5, 65536), (3, 40000), (32, 9000)):
    bufs = [m.DeviceBuffer(nb * 4096) for _ in range(Q)]
    for i, b in enumerate(bufs):
        b.upload(synth.splitmix_bytes(0xC0FFEE + 77 * i + nb, nb * 4096))
    ref = []
    for b in bufs:
        o = m.DeviceBuffer(nb * 4)
        eng.batch_uniform(b, nb, 4096, 4096, o)
        ref.append(o)
    outs = [m.DeviceBuffer(nb * 4) for _ in range(Q)]
    jobs = m.ujobs([(bufs[i], nb, outs[i]) for i in range(Q)])
    for rep in range(4):
        for o in outs:
            o.upload(np.zeros(nb * 4, np.uint8))
        eng.batch_uniform_queue(jobs, 4096, 4096)
        eng.sync()
        for i in range(Q):
            a = np.frombuffer(outs[i].download(), np.uint32)
            r = np.frombuffer(ref[i].download(), np.uint32)
            assert (a == r).all(), (Q, nb, rep, i, int((a != r).sum()))
    print("ok", Q, nb)
