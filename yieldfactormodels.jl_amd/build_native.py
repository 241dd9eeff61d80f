"""Build libyfm_hip.so (gfx950) in-tree with hipcc — no torch, no JIT cache.

Called by ``__graft_entry__.build()``.  Each translation unit is compiled to an
object in ``build/`` in parallel, then linked into ``yfm_amd/libyfm_hip.so``.
A rebuild happens only when a source or header is newer than the library.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "build"
LIB = PKG / "yfm_amd" / "libyfm_hip.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("YFM_OFFLOAD_ARCH", "gfx950")
# -amdgpu-spill-vgpr-to-agpr=0: register spills go to scratch memory, never to AGPRs.  ROCm 7.2's backend
# miscompiles the VGPR->AGPR spill path of the heavily spilling fixed-loading instantiations (GNS5 NP = 48,
# ~850 spilled VGPRs): the same filter written as two functions returned O(1)-wrong logliks there, while
# the host build of the same C++ is MemorySanitizer-clean and bitwise equal in both forms
# (tools/host_fixedz/; tests/test_gpu_split_form.py).  Only the 12 spilling kernels change;
# the config 2-5 kernels are byte-identical either way.
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-mllvm", "-amdgpu-spill-vgpr-to-agpr=0", f"-I{ROOT / 'include'}"]


def _sources():
    return sorted(CSRC.glob("*.hip"))


def _deps():
    return list(CSRC.glob("*")) + list((ROOT / "include").glob("*.h")) + [Path(__file__)]


STAMP = BUILD / "flags.stamp"


def _stamp() -> str:
    """The compiler, target and flags the objects in build/ were made with: a different stamp forces a full
    rebuild (objects for another arch or flag set must never be linked together)."""
    return "\n".join([HIPCC, ARCH, *FLAGS]) + "\n"


def _stamp_ok() -> bool:
    return STAMP.exists() and STAMP.read_text() == _stamp()


def up_to_date() -> bool:
    if not LIB.exists() or not _stamp_ok():
        return False
    t = LIB.stat().st_mtime
    return all(p.stat().st_mtime <= t for p in _deps())


def build(force: bool = False, verbose: bool = True) -> Path:
    if not force and up_to_date():
        return LIB
    BUILD.mkdir(exist_ok=True)
    if not _stamp_ok():
        force = True
    srcs = _sources()
    objs = [BUILD / (s.stem + ".o") for s in srcs]

    def cc(pair):
        s, o = pair
        cmd = [HIPCC, *FLAGS, "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    # an object is rebuilt when it is older than its source, a header or this script (a header change
    # rebuilds everything: the headers are shared by most translation units)
    hdr = max([p.stat().st_mtime for p in CSRC.glob("*.hpp")] + [p.stat().st_mtime for p in (ROOT / "include").glob("*.h")]
              + [Path(__file__).stat().st_mtime])
    todo = [(s, o) for s, o in zip(srcs, objs)
            if force or not o.exists() or o.stat().st_mtime < max(s.stat().st_mtime, hdr)]
    # a half-finished rebuild (a failed compile or link) must not pass as the stamped one: the stamp goes now and
    # is written back only after the link succeeded, so the library beside it was made with these flags
    STAMP.unlink(missing_ok=True)
    with ThreadPoolExecutor(max_workers=max(1, min(len(todo), 4))) as ex:
        list(ex.map(cc, todo))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(LIB)]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    STAMP.write_text(_stamp())
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
