"""Time the general path (lcrc_batch_uniform with length != stride or != 4096) for a few shapes, on the
library named by LCRC_LIB_PATH and the general-path kernel named by argv[1] (auto | ranges | blocks: the context
option `general`, lcrc_ctx_create_ex; the library reads no environment variable)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
buf = m.DeviceBuffer.from_host(synth.splitmix_bytes(7, 300 << 20))
out = m.DeviceBuffer(4 * 70000)
GENERAL = sys.argv[1] if len(sys.argv) > 1 else "auto"
eng = m.Engine(0, m.MODE_C, general=GENERAL)
eng.reserve(300 << 20)
for length, stride in [(4096, 4100), (4096, 4096 + 4096), (4000, 4004), (2048, 2052), (512, 516), (65536, 65540),
                       (4092, 4096), (4097, 4101)]:
    n = min(65536, (256 << 20) // stride)
    for _ in range(3):
        eng.batch_uniform(buf, n, length, stride, out)
    eng.sync()
    eng.timer_start()
    for _ in range(10):
        eng.batch_uniform(buf, n, length, stride, out)
    ms = eng.timer_stop() / 10
    print(f"{GENERAL}: len {length:6d} stride {stride:6d} n {n:6d}: "
          f"{ms * 1e3:8.1f} us  {n * length / ms / 1e6:8.1f} GB/s", flush=True)
# the same shapes as descriptors (lcrc_batch), without and with an expected value
for length, stride in [(4096, 4100), (4097, 4101), (4000, 4004)]:
    n = min(65536, (256 << 20) // stride)
    for xr in (None, length):
        d = np.zeros(n, m.DESC_DTYPE)
        d["offset"] = np.arange(n, dtype=np.uint64) * stride
        d["length"] = length
        d["expect_rel"] = m.NO_EXPECT if xr is None else xr
        dd = m.DeviceBuffer.from_host(d.view(np.uint8))
        for _ in range(3):
            eng.batch(buf, 300 << 20, dd, n, out)
        eng.sync()
        eng.timer_start()
        for _ in range(10):
            eng.batch(buf, 300 << 20, dd, n, out)
        ms = eng.timer_stop() / 10
        print(f"{GENERAL}: descs len {length} stride {stride} expect {xr}: "
              f"{ms * 1e3:8.1f} us", flush=True)
