"""Build libdragg_mi355x.so in-tree for gfx950 (hipcc).  `python -m dragg_amd.build`.

The library carries the sha-256 of its sources (the kernel file and the C header) as a stamp
(`dragg_mpc_source_hash()`, also findable in the file's bytes after STAMP_PREFIX): `needs_build()`
rebuilds whenever the stamp differs from the sources on disk (file times alone lie after a
checkout), and `dragg_amd._lib.load()` refuses a library whose stamp is not the sources'.
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = [os.path.join(HERE, "csrc", "mpc_kernel.hip")]
HEADER = os.path.join(HERE, "..", "include", "dragg_mi355x.h")
OUT = os.path.join(HERE, "libdragg_mi355x.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# iterative-ilp machine scheduling: +1 % on the bench workload over the default (A/B in
# DESIGN.md section 5; scheduling reorders instructions only, the results are bit-identical)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall",
         "-Wno-unused-function", "-Wno-unused-variable", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
STAMP_PREFIX = b"dragg-source-sha256:"


def source_hash(srcs=None):
    """sha-256 over the sources the library is built from (kernel file(s), then the header)."""
    h = hashlib.sha256()
    for p in list(srcs or SRC) + [HEADER]:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def stamp_of(lib_path):
    """The source stamp inside a built library file (None: none found)."""
    try:
        with open(lib_path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(STAMP_PREFIX)
    if i < 0:
        return None
    j = i + len(STAMP_PREFIX)
    return data[j:j + 64].decode("ascii", "replace")


def sources_present():
    return all(os.path.exists(p) for p in SRC + [HEADER])


def needs_build():
    if not os.path.exists(OUT):
        return True
    return sources_present() and stamp_of(OUT) != source_hash()


def build(force=False, verbose=False):
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC] + FLAGS + [f'-DDRAGG_SOURCE_HASH="{source_hash()}"', "-o", OUT] + SRC
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({' '.join(cmd)}):\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(r.stderr, file=sys.stderr)
    return OUT


# the host-side results formatter (include/dragg_results.h): g++, OpenMP, no GPU code
RES_SRC = [os.path.join(HERE, "csrc", "results_writer.cpp")]
RES_HEADER = os.path.join(HERE, "..", "include", "dragg_results.h")
RES_OUT = os.path.join(HERE, "libdragg_results.so")
RES_PREFIX = b"dragg-results-sha256:"


def results_hash():
    h = hashlib.sha256()
    for p in RES_SRC + [RES_HEADER]:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stamp(lib_path, prefix):
    try:
        with open(lib_path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(prefix)
    return None if i < 0 else data[i + len(prefix):i + len(prefix) + 64].decode("ascii", "replace")


def results_needs_build():
    if not os.path.exists(RES_OUT):
        return True
    return all(os.path.exists(p) for p in RES_SRC + [RES_HEADER]) and _stamp(RES_OUT, RES_PREFIX) != results_hash()


def build_results(force=False):
    """libdragg_results.so (seconds: one small C++ file)."""
    if not force and not results_needs_build():
        return RES_OUT
    tmp = RES_OUT + f".{os.getpid()}.tmp"
    cmd = [os.environ.get("CXX", "g++"), "-O3", "-std=c++17", "-fopenmp", "-shared", "-fPIC", "-Wall",
           f'-DDRAGG_RESULTS_SOURCE_HASH="{results_hash()}"', "-o", tmp] + RES_SRC
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"g++ failed ({' '.join(cmd)}):\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, RES_OUT)                  # (atomic: concurrent processes never load a half-written file)
    return RES_OUT


if __name__ == "__main__":
    build_results(force="--force" in sys.argv)
    print(build(force="--force" in sys.argv, verbose=True))
