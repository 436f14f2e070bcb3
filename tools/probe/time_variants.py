"""Times the 4 KiB fast path of each ablation build (LCRC_LIB_PATH per subprocess)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import os, sys
sys.path.insert(0, ROOT)
import __graft_entry__ as g
m = g.load()
NB = 65536; BUFS = 4
bufs = [m.DeviceBuffer(NB * 4096) for _ in range(BUFS)]
for i, b in enumerate(bufs):
    b.upload(__import__("leveldb_rust_amd.synth", fromlist=["x"]).splitmix_bytes(0x5EED0001 + i, NB * 4096))
out = m.DeviceBuffer(NB * 4)
eng = m.Engine(0, 1)
res = []
for rep in range(3):
    for i in range(5):
        eng.batch_uniform(bufs[i % BUFS], NB, 4096, 4096, out)
    eng.timer_start()
    for i in range(100):
        eng.batch_uniform(bufs[i % BUFS], NB, 4096, 4096, out)
    res.append(eng.timer_stop() / 100)
ms = min(res)
clk = ""
if hasattr(m.lib(), "lcrc_probe_clock_mhz"):
    import ctypes
    f = m.lib().lcrc_probe_clock_mhz
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_int]
    clk = f"  clock {f(256):.0f} MHz"
print(f"{os.path.basename(os.environ['LCRC_LIB_PATH']):18s} {ms*1000:7.1f} us  {NB*4096/ms/1e6:7.1f} GB/s{clk}")
'''.replace("ROOT", repr(ROOT))
vdir = os.path.join(ROOT, "tools", "probe", "variants")
for v in sys.argv[1:] or sorted(os.listdir(vdir)):
    env = dict(os.environ, LCRC_LIB_PATH=os.path.join(vdir, v if v.endswith(".so") else v + ".so"))
    subprocess.run([sys.executable, "-c", CHILD], env=env, check=False, timeout=120)
