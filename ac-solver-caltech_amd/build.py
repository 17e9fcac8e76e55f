"""Build libacx.so in-tree: hipcc --offload-arch=gfx950 (cross-compiles without a GPU).

    python ac-solver-caltech_amd/build.py [--force]

The library links only the HIP runtime (soname libamdhip64.so.7); when it is loaded after
`import torch` the dynamic linker binds it to the runtime torch already mapped, so device
pointers and streams from torch are valid in it.  No torch headers are used.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "acx", "libacx.so")
INCLUDE = os.path.join(REPO, "include")
SOURCES = ["acx_kernels.hip", "acx_bfs.hip", "acx_sbfs.hip", "acx_features.hip", "acx_curriculum.hip", "acx_words.hip",
           "acx_greedy.hip", "acx_search.cpp"]
# acx_kernels.hip is also compiled once per instantiation part (-DACX_PART=n, see the file's
# "extern template" block), in parallel: the runtime-L generic sets took ~7 minutes in one object
KERNEL_PARTS = 10
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ACX_OFFLOAD_ARCH", "gfx950")


def source_files() -> list:
    """Every file the library is compiled from, in a fixed order (the provenance hash's input)."""
    files = [os.path.join(CSRC, s) for s in SOURCES]
    files += sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hpp")))
    return files + [os.path.join(INCLUDE, "acx.h"), os.path.abspath(__file__)]


def source_hash() -> str:
    """sha256 over the names and contents of source_files(); built into acx_version() as
    "src:<hash>" so a library that was not compiled from the shipped sources is detected
    (__graft_entry__.smoke() and tests/test_cpu_host.py compare the two)."""
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


MARK = b"acx-src-sha256:"


def built_hash(path: str = OUT):
    """the source hash embedded in a built library (None if absent)"""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as fh:
        data = fh.read()
    i = data.find(MARK)
    return data[i + len(MARK): i + len(MARK) + 64].decode("ascii", "replace") if i >= 0 else None


def _stale() -> bool:
    return built_hash() != source_hash()


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    digest = source_hash()
    objs = []
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    procs = []
    headers = [os.path.join(INCLUDE, "acx.h")] + [os.path.join(CSRC, f) for f in os.listdir(CSRC)
                                                   if f.endswith((".h", ".hpp"))]
    units = [(src, None) for src in SOURCES] + [("acx_kernels.hip", n) for n in range(1, KERNEL_PARTS + 1)]
    for src, part in units:
        obj = os.path.join(HERE, "build", src + (f".p{part}" if part else "") + ".o")
        objs.append(obj)
        main_kernels = src == "acx_kernels.hip" and part is None  # carries the source hash: always rebuilt
        if not force and os.path.exists(obj) and not main_kernels:
            t = os.path.getmtime(obj)
            if all(os.path.getmtime(d) <= t for d in [os.path.join(CSRC, src), __file__] + headers):
                continue  # object up to date
        if src.endswith(".hip"):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", "-I", INCLUDE,
                   "-Wno-pass-failed", f'-DACX_SOURCE_HASH="{digest}"', os.path.join(CSRC, src), "-o", obj]
            if part:  # no source hash in the parts: acx_version() is in the main object
                cmd = [c for c in cmd if not c.startswith("-DACX_SOURCE_HASH")]
                cmd.insert(-3, f"-DACX_PART={part}")
        else:
            cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-c", "-I", INCLUDE, os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("libacx build failed")
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT] + objs
    if verbose:
        print(" ".join(link))
    subprocess.check_call(link)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args()
    print(build(force=args.force, verbose=args.verbose))
    sys.exit(0)
