"""Runs the 4 KiB fast path N times with the library named by LCRC_LIB_PATH (for rocprofv3)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
NB = 65536
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 1
bufs = [m.DeviceBuffer(NB * 4096) for _ in range(4)]
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
for i, b in enumerate(bufs):
    b.upload(synth.splitmix_bytes(0x5EED0001 + i, NB * 4096))
out = m.DeviceBuffer(NB * 4)
eng = m.Engine(0, mode)
for i in range(iters):
    eng.batch_uniform(bufs[i % 4], NB, 4096, 4096, out)
eng.sync()
print("done")
