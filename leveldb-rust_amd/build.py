"""Build the in-tree shared library `_build/liblcrc.so` (HIP kernels for gfx950 + C ABI + C++ host
restatement) with hipcc. No JIT cache, no site-packages install: the .so lives next to this file so it
travels to the GPU box with the repository snapshot."""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "liblcrc.so")
SOURCES = ["lcrc_kernels.hip", "lcrc_api.cpp", "lcrc_scalar.cpp", "lcrc_leveldb.cpp", "lcrc_table.cpp", "lcrc_tbuild.cpp"]
HEADERS = ["lcrc_device.h", "lcrc_math.h", "lcrc_table.h", os.path.join("..", "..", "include", "lcrc.h")]
ARCH = os.environ.get("LCRC_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def source_hash(extra_flags=()):
    """sha256 (16 hex digits) of every source and header the library is built from, of this recipe and of any
    extra compile flags. It is compiled into lcrc_version(), so a library can be matched to the tree and the
    flags it claims to come from: smoke() checks the loaded library against the tree it runs in with NO extra
    flags, so a library built with any define of its own fails that check."""
    h = hashlib.sha256()
    for name in sorted(SOURCES + HEADERS) + [os.path.basename(__file__)]:
        path = __file__ if name == os.path.basename(__file__) else os.path.join(CSRC, name)
        h.update(name.encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
    for flag in extra_flags:
        h.update(b"flag\0" + flag.encode() + b"\0")
    return h.hexdigest()[:16]


def _stale():
    """Rebuild unless the library carries this tree's source hash (mtimes do not survive a copy)."""
    if not os.path.exists(LIB):
        return True
    with open(LIB, "rb") as f:
        return ("src " + source_hash()).encode() not in f.read()


def build(force=False, verbose=False, extra_flags=()):
    """The in-tree library. Diagnostic builds (-DLCRC_PROBE_*: clock stamps) go to tools/probe/variants via
    tools/probe/build_one.sh, never here."""
    extra_flags = tuple(extra_flags)
    bad = [f for f in extra_flags if f.replace(" ", "").startswith("-DLCRC_PROBE")]
    if bad:
        raise ValueError(f"build.py: {bad} are diagnostic flags; the in-tree library is built without them")
    if not force and not extra_flags and not _stale():
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    # the atomic optimizer would read the ticket atomic's result at once (readfirstlane + vmcnt(0)),
    # stalling on every load issued before it; k_windows reads it one walk later instead
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
           "-Wall", "-Wno-unused-result", f'-DLCRC_SRC_HASH="{source_hash(extra_flags)}"', "-o", tmp] + list(extra_flags) + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
