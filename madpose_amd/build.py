"""Build the MI355X engine library in-tree: madpose_amd/lib/libmadpose_mi355x.so.

hipcc cross-compiles for gfx950 without a GPU.  Every translation unit is built as
HIP (host + device); the shared library exports the C ABI of
include/madpose_mi355x.h.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(HERE, "lib", "obj")
LIB = os.path.join(LIBDIR, "libmadpose_mi355x.so")

SOURCES = [
    os.path.join(CSRC, "kernels", "kernels.hip"),
    os.path.join(CSRC, "host", "engine.cpp"),
    os.path.join(CSRC, "capi.cpp"),
]
# host-only translation units (plain C++, no device pass): the LO sweep carries an
# AVX-512 function beside its x86-64-v3 baseline, chosen at run time (host/lo_sweep.cpp)
HOST_SOURCES = [
    os.path.join(CSRC, "host", "lo_sweep.cpp"),
    os.path.join(CSRC, "host", "lm.cpp"),
    os.path.join(CSRC, "host", "lm_eval_w4.cpp"),
    os.path.join(CSRC, "host", "lm_eval_w8.cpp"),
]
# per-file host flags: the AVX-512 build of the LM's residual evaluation (chosen at run
# time, host/lm.cpp lm_eval_avx512)
HOST_EXTRA = {os.path.join(CSRC, "host", "lm_eval_w8.cpp"): ["-march=x86-64-v4"]}
HEADERS = [
    os.path.join(dp, f)
    for dp, _, fs in os.walk(CSRC)
    for f in fs
    if f.endswith(".h") or f.endswith(".inc")
] + [os.path.join(ROOT, "include", "madpose_mi355x.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HOSTCXX = os.environ.get("MADPOSE_HOSTCXX", "/opt/rocm/llvm/bin/clang++")
HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-I", os.path.join(ROOT, "include"), "-Wall", "-Wno-unused-function",
              "-march=x86-64-v3", "-mprefer-vector-width=512"]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include"), "-Wall",
         "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-result",
         # host side only: AVX2/FMA for the 4-wide LM residual loop (lm.cpp); the
         # device side stays plain gfx950
         "-Xarch_host", "-march=x86-64-v3"]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    if _newer(obj, [src, __file__] + HEADERS):
        if src in HOST_SOURCES:
            cmd = [HOSTCXX] + HOST_FLAGS + HOST_EXTRA.get(src, []) + ["-c", src, "-o", obj]
        else:
            cmd = [HIPCC, "-x", "hip"] + FLAGS + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return obj


def build_library(verbose=False):
    os.makedirs(OBJDIR, exist_ok=True)
    with ThreadPoolExecutor(max_workers=4) as ex:
        objs = list(ex.map(_compile, SOURCES + HOST_SOURCES))
    if _newer(LIB, objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB] + objs + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build_library(verbose=True)
    sys.exit(0)
