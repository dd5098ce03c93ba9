"""Build libofl_codec.so (gfx950) in-tree with hipcc.

The library is a plain C-ABI shared object (include/ofl_codec.h); it is loaded
with ctypes by openfl_amd._lib and never links against torch.  Output:
openfl_amd/lib/libofl_codec.so (git-ignored; travels to the GPU box with the
repo snapshot).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libofl_codec.so")
SOURCES = ["eden_kernels.hip", "lossy_kernels.hip", "agg_kernels.hip", "deflate_kernels.hip", "serial_sum.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-std=c++20", "-O3", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def _stale():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(ROOT, "include", "ofl_codec.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not _stale():
        return LIB_PATH
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB_PATH + ".tmp"
    cmd = [HIPCC] + FLAGS + ["-o", tmp] + [os.path.join(CSRC, s) for s in SOURCES] + ["-lz"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
