"""Times the queued 4 KiB fast path (lcrc_batch_uniform_queue, 20 x 256 MiB batches per launch, 4 rotating
buffers) of each build in tools/probe/variants/q_*.so (LCRC_LIB_PATH per subprocess): microseconds per batch."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import os, sys
sys.path.insert(0, ROOT)
import __graft_entry__ as g
m = g.load()
NB = 65536; BUFS = 4; Q = 20
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
bufs = [m.DeviceBuffer.from_host(synth.splitmix_bytes(0x5EED0001 + i, NB * 4096)) for i in range(BUFS)]
outs = [m.DeviceBuffer(NB * 4) for _ in range(BUFS)]
eng = m.Engine(0, 1, 1)
jobs = m.ujobs([(bufs[i % BUFS], NB, outs[i % BUFS]) for i in range(Q)])
eng.batch_uniform_queue(jobs, 4096, 4096)
eng.sync()
res = []
for rep in range(5):
    eng.timer_start()
    eng.batch_uniform_queue(jobs, 4096, 4096)
    res.append(eng.timer_stop() / Q)
    eng.sync()
ms = sorted(res)[len(res) // 2]
clk = ""
if hasattr(m.lib(), "lcrc_probe_clock_mhz"):  # LCRC_PROBE_CLOCK builds: median workgroup shader clock
    import ctypes
    f = m.lib().lcrc_probe_clock_mhz
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_int]
    clk = f"  clock {f(256):.0f} MHz"
print(f"{os.path.basename(os.environ['LCRC_LIB_PATH']):18s} {ms*1000:7.2f} us/batch  {NB*4096/ms/1e6:7.1f} GB/s  "
      f"frac {NB*4096/ms/1e6/8000:.4f}  (min {min(res)*1000:.2f}, max {max(res)*1000:.2f}){clk}", flush=True)
'''.replace("ROOT", repr(ROOT))
vdir = os.path.join(ROOT, "tools", "probe", "variants")
names = sys.argv[1:] or sorted(f for f in os.listdir(vdir) if f.startswith("q_"))
for v in names:
    env = dict(os.environ, LCRC_LIB_PATH=os.path.join(vdir, v if v.endswith(".so") else v + ".so"))
    subprocess.run([sys.executable, "-c", CHILD], env=env, check=False, timeout=120)
