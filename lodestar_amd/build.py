"""Build the gfx950 HIP library in-tree (lodestar_amd/libgbv.so) with hipcc."""
import os
import subprocess
import sys

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


def _compile(src, obj, verbose):
    cmd = ["hipcc", "--offload-arch=%s" % ARCH, "-O3", "-fPIC", "-std=c++17", "-c", src, "-o", obj + ".tmp"]
    cmd[1:1] = os.environ.get("GBV_EXTRA_CFLAGS", "").split()  # experiments only (e.g. -mllvm options)
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(obj + ".tmp", obj)
    return obj


def build(force=False, verbose=False, jobs=None):
    """Compile each kernel family (lodestar_amd/csrc/*.hip) in parallel and link libgbv.so.

    Serialised across processes with a file lock (bench.py ranks all call it): the first caller
    builds, the others find the library fresh once they hold the lock."""
    if not force and not needs_build():
        return LIB
    import fcntl
    with open(os.path.join(HERE, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and not needs_build():
            return LIB
        return _build_locked(force, verbose, jobs)


def _build_locked(force, verbose, jobs):
    from concurrent.futures import ThreadPoolExecutor
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    tus = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith(".hip")]
    headers_t = max(os.path.getmtime(s) for s in sources() if not s.endswith(".hip"))
    jobs = jobs or min(len(tus), max(1, (os.cpu_count() or 4)))
    todo = []
    objs = []
    for src in tus:
        obj = os.path.join(objdir, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(headers_t, os.path.getmtime(src)):
            todo.append((src, obj))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda t: _compile(t[0], t[1], verbose), todo))
    cmd = ["hipcc", "--offload-arch=%s" % ARCH, "-shared", "-fPIC", "-o", LIB + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    import time
    t = time.time()
    build(force="--force" in sys.argv, verbose=True)
    print("built", LIB, "in %.1fs" % (time.time() - t))
