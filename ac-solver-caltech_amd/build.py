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


HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wno-pass-failed"]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC"]


def toolchain_id() -> str:
    """what else decides the machine code: the offload arch, the compilers and their flags"""
    return "|".join([ARCH, os.path.realpath(HIPCC), " ".join(HIP_FLAGS), "g++", " ".join(CXX_FLAGS),
                     f"parts={KERNEL_PARTS}"])


def source_hash() -> str:
    """sha256 over the names and contents of source_files() and the toolchain (arch, compilers,
    flags); built into acx_version() as "src:<hash>" so a library that was not compiled from the
    shipped sources for this arch is detected (__graft_entry__.smoke() and tests/test_cpu_host.py
    compare the two)."""
    h = hashlib.sha256()
    h.update(toolchain_id().encode() + b"\0")
    for f in source_files():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


MARK = b"acx-src-sha256:"
STAMP = OUT + ".stamp"  # sidecar: the hash the library next to it was built with (written after the link)


def built_hash(path: str = OUT):
    """the source hash embedded in a built library (None if absent): read from the library in
    1 MiB windows (no whole-file read)"""
    if not os.path.exists(path):
        return None
    win, tail = 1 << 20, b""
    with open(path, "rb") as fh:
        while True:
            chunk = fh.read(win)
            if not chunk:
                return None
            data = tail + chunk
            i = data.find(MARK)
            if i >= 0:
                rest = data[i + len(MARK):]
                if len(rest) < 64:
                    rest += fh.read(64)
                return rest[:64].decode("ascii", "replace")
            tail = data[-(len(MARK) + 64):]


def _stale(digest: str) -> bool:
    """the library is up to date when its sidecar stamp (or, without one, its embedded hash)
    matches `digest`"""
    if not os.path.exists(OUT):
        return True
    if os.path.exists(STAMP) and os.path.getmtime(STAMP) >= os.path.getmtime(OUT):
        with open(STAMP) as f:
            return f.read().strip() != digest
    return built_hash() != digest


def _obj_stamp(obj: str) -> str:
    return obj + ".tc"  # the toolchain an object was compiled with


def build(force: bool = False, verbose: bool = False) -> str:
    digest = source_hash()
    if not force and not _stale(digest):
        return OUT
    tc = toolchain_id()
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
        if not force and os.path.exists(obj) and not main_kernels and os.path.exists(_obj_stamp(obj)):
            t = os.path.getmtime(obj)
            with open(_obj_stamp(obj)) as f:
                same_tc = f.read() == tc
            if same_tc and all(os.path.getmtime(d) <= t for d in [os.path.join(CSRC, src), __file__] + headers):
                continue  # object up to date, same arch / compiler / flags
        if src.endswith(".hip"):
            cmd = [HIPCC, f"--offload-arch={ARCH}", *HIP_FLAGS, "-c", "-I", INCLUDE,
                   f'-DACX_SOURCE_HASH="{digest}"', os.path.join(CSRC, src), "-o", obj]
            if part:  # no source hash in the parts: acx_version() is in the main object
                cmd = [c for c in cmd if not c.startswith("-DACX_SOURCE_HASH")]
                cmd.insert(-3, f"-DACX_PART={part}")
        else:
            cmd = ["g++", *CXX_FLAGS, "-c", "-I", INCLUDE, os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((obj, subprocess.Popen(cmd)))
    for obj, p in procs:
        if p.wait() != 0:
            raise RuntimeError("libacx build failed")
        with open(_obj_stamp(obj), "w") as f:
            f.write(tc)
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT] + objs
    if verbose:
        print(" ".join(link))
    subprocess.check_call(link)
    with open(STAMP, "w") as f:
        f.write(digest)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args()
    print(build(force=args.force, verbose=args.verbose))
    sys.exit(0)
