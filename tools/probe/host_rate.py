"""Host submission cost of one batch_uniform call vs its GPU time (is the bench host-bound?)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
NB = 65536
bufs = [m.DeviceBuffer(NB * 4096) for _ in range(4)]
for i, b in enumerate(bufs):
    b.upload(synth.splitmix_bytes(0x5EED0001 + i, NB * 4096))
engs = [m.Engine(0, 1, 1) for _ in range(2)]
outs = [m.DeviceBuffer(NB * 4) for _ in range(2)]
for nb in (16, NB):
    for S in (1, 2):
        for e in engs:
            e.sync()
        K = 200
        t0 = time.perf_counter()
        for i in range(K):
            engs[i % S].batch_uniform(bufs[i % 4], nb, 4096, 4096, outs[i % S])
        t1 = time.perf_counter()
        for e in engs:
            e.sync()
        t2 = time.perf_counter()
        print(f"nblk {nb:6d} streams {S}: submit {(t1 - t0) / K * 1e6:6.1f} us/step, total {(t2 - t0) / K * 1e6:6.1f} us/step")
