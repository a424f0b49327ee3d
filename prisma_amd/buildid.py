"""Build provenance of libprisma_amd.so.

The build id is a hash of every source the library is compiled from plus the
compiler flags.  `__graft_entry__.build_engine` compiles it into the library
(`-DPRISMA_BUILD_ID=...`, exported as `prisma_build_id()`), `engine.load_library`
refuses a library whose id differs from the tracked sources, and bench.py prints
it and keys the committed PMC traffic figures on it.  No torch import here.
"""
from __future__ import annotations

import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "prisma_amd", "csrc")

ENGINE_SOURCES = ["prisma_engine.hip", "prisma_engine_mlp.hip", "prisma_engine_lite.hip", "prisma_engine_lite_mlp.hip",
                  "prisma_engine_mem.hip"]
ENGINE_HEADERS = ["engine_core.h", "engine_layout.h", "numerics.h", "step_kernel.h", "mrg32k3a.h"]
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fPIC", "-std=c++17",
               # the per-replica counters are bumped by lane 0 only: the atomic optimizer's
               # wave-aggregation rewrite (mbcnt, bcnt, exec juggling per add) is pure overhead
               "-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]
MARKER = b"PRISMA_BUILD_ID="


def source_files() -> list:
    return ([os.path.join(CSRC, f) for f in ENGINE_SOURCES + ENGINE_HEADERS]
            + [os.path.join(ROOT, "include", "prisma.h")])


def source_hash(extra_flags=()) -> str:
    """12 hex digits over the kernel/ABI sources and the compile flags."""
    h = hashlib.sha1()
    for f in source_files():
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode() + b"\0" + fh.read() + b"\0")
    h.update(" ".join(list(HIPCC_FLAGS) + list(extra_flags)).encode())
    return h.hexdigest()[:12]


def sources_present() -> bool:
    return all(os.path.exists(f) for f in source_files())


def embedded_id(lib_path: str):
    """The build id compiled into a library file (read from its bytes, no dlopen), or None."""
    try:
        with open(lib_path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    i = data.find(MARKER)
    if i < 0:
        return None
    return data[i + len(MARKER): i + len(MARKER) + 12].decode(errors="replace")
