"""Build the gfx950 HIP library in-tree (lodestar_amd/libgbv.so) with hipcc."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgbv.so")
ARCH = os.environ.get("GBV_OFFLOAD_ARCH", "gfx950")


def sources():
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith((".h", ".hip"))] + [
        os.path.join(ROOT, "include", "gbv.h")]


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in sources())


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    cmd = ["hipcc", "--offload-arch=%s" % ARCH, "-O3", "-fPIC", "-shared", "-std=c++17",
           "-o", LIB + ".tmp", os.path.join(CSRC, "gbv.hip")]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force=True, verbose=True)
    print("built", LIB)
