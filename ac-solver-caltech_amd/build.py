"""Build libacx.so in-tree: hipcc --offload-arch=gfx950 (cross-compiles without a GPU).

    python ac-solver-caltech_amd/build.py [--force]

The library links only the HIP runtime (soname libamdhip64.so.7); when it is loaded after
`import torch` the dynamic linker binds it to the runtime torch already mapped, so device
pointers and streams from torch are valid in it.  No torch headers are used.
"""
from __future__ import annotations

import argparse
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
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ACX_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(INCLUDE, "acx.h"), __file__]
    deps += [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hpp"))]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    objs = []
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    procs = []
    headers = [os.path.join(INCLUDE, "acx.h")] + [os.path.join(CSRC, f) for f in os.listdir(CSRC)
                                                   if f.endswith((".h", ".hpp"))]
    for src in SOURCES:
        obj = os.path.join(HERE, "build", src + ".o")
        objs.append(obj)
        if not force and os.path.exists(obj):
            t = os.path.getmtime(obj)
            if all(os.path.getmtime(d) <= t for d in [os.path.join(CSRC, src), __file__] + headers):
                continue  # object up to date
        if src.endswith(".hip"):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", "-I", INCLUDE,
                   "-Wno-pass-failed", os.path.join(CSRC, src), "-o", obj]
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
