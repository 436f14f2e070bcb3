"""Sparse verify (lcrc_batch_covered) shapes: where the per-call time goes. Run under
rocprofv3 --kernel-trace -d DIR -o run, then tools/probe/kernel_times.py DIR/run_results.db."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
eng = m.Engine(0, m.MODE_C)
big = m.DeviceBuffer(1 << 30)
small = m.DeviceBuffer(16 << 20)
out, mm = m.DeviceBuffer(4096), m.DeviceBuffer(512)
rng = np.random.default_rng(5)


def case(name, buf, size, offs, lens, reps=20):
    d = np.zeros(len(offs), m.DESC_DTYPE)
    d["offset"], d["length"], d["expect_rel"] = offs, lens, lens
    dd = m.DeviceBuffer.from_host(d.view(np.uint8))
    cov = int(np.asarray(lens, np.uint64).sum())
    for _ in range(3):
        eng.batch(buf, size, dd, len(offs), out, mm, covered=cov)
    eng.sync()
    eng.timer_start()
    for _ in range(reps):
        eng.batch(buf, size, dd, len(offs), out, mm, covered=cov)
    us = eng.timer_stop() / reps * 1e3
    print(f"{name:48s} {us:7.2f} us per call", flush=True)


sp = np.sort(rng.choice((1 << 30) // 8192 - 1, 100, replace=False)).astype(np.uint64) * 8192
case("1 GiB, 100 x 4097 B, random offsets", big, 1 << 30, sp + rng.integers(0, 4000, 100).astype(np.uint64),
     np.full(100, 4097, np.uint32))
case("1 GiB, 100 x 4092 B, 4 KiB-aligned", big, 1 << 30, sp, np.full(100, 4092, np.uint32))
case("1 GiB, 100 x 200 B", big, 1 << 30, sp, np.full(100, 200, np.uint32))
case("1 GiB, 1 x 4092 B", big, 1 << 30, sp[:1], np.full(1, 4092, np.uint32))
case("16 MiB, 100 x 4097 B, back to back", small, 16 << 20, np.arange(100, dtype=np.uint64) * 8192 + 3,
     np.full(100, 4097, np.uint32))
case("16 MiB, 100 x 4092 B, back to back", small, 16 << 20, np.arange(100, dtype=np.uint64) * 4096,
     np.full(100, 4092, np.uint32))
case("16 MiB, 1000 x 4092 B", small, 16 << 20, np.arange(1000, dtype=np.uint64) * 8192 % (16 << 20),
     np.full(1000, 4092, np.uint32))
eng.close()
