"""Build the in-tree shared library `_build/liblcrc.so` (HIP kernels for gfx950 + C ABI + C++ host
restatement) with hipcc. No JIT cache, no site-packages install: the .so lives next to this file so it
travels to the GPU box with the repository snapshot."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "liblcrc.so")
SOURCES = ["lcrc_kernels.hip", "lcrc_api.cpp", "lcrc_scalar.cpp", "lcrc_leveldb.cpp", "lcrc_table.cpp"]
HEADERS = ["lcrc_device.h", "lcrc_math.h", "lcrc_table.h", os.path.join("..", "..", "include", "lcrc.h")]
ARCH = os.environ.get("LCRC_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False, extra_flags=()):
    if not force and not _stale():
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    # the atomic optimizer would read the ticket atomic's result at once (readfirstlane + vmcnt(0)),
    # stalling on every load issued before it; k_windows reads it one walk later instead
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
           "-Wall", "-Wno-unused-result", "-o", tmp] + list(extra_flags) + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
