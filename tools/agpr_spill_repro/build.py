"""Build the reproducer of the ROCm 7.2 VGPR→AGPR spill miscompile on the CPU.

The miscompile was seen in the sources of commit 13e51a6 (the last build without the fence; the diagnosis is
commit 2a12bbb, profiles/r4/diag1/).  This script extracts that revision's kernel sources with `git archive`
(this repository's own history) and builds, from the SAME sources and the flags of
yieldfactormodels.jl_amd/build_native.py, two libraries that differ only in the fence
`-mllvm -amdgpu-spill-vgpr-to-agpr=0`:

    build/libyfm_13e51a6_fenced.so     build/libyfm_13e51a6_unfenced.so

plus `repro` (host C++, dlopen's a library and runs case2431.bin in both update forms) and
build/spill_report.txt: for the two-function NP = 48 GNS5 kernel, the AGPR moves and scratch accesses of each
build's device assembly, and the same for HEAD's sources (whose kernel compiles identically with and without
the fence since the round-4 setup changes — the fence stays because nothing guarantees that for the next
change or compiler).  Run `tools/agpr_spill_repro/run.sh` on a GPU box afterwards."""
from __future__ import annotations

import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT / "yieldfactormodels.jl_amd"))
import build_native as BN  # noqa: E402

REV = "13e51a6"
OUT = HERE / "build"
FENCE = ["-mllvm", "-amdgpu-spill-vgpr-to-agpr=0"]
KERNEL = "_ZN3yfm20fixedz_loglik_kernelILi48ELi5ELi2ELb0ELb0ELb1E"  # <48, 5, 2, RECORD=0, STEADY=0, SPLIT_FORM=1>


def unfenced(flags):
    i = next(k for k in range(len(flags) - 1) if flags[k:k + 2] == FENCE)
    return flags[:i] + flags[i + 2:]


def with_include(flags, inc: Path):
    return [f"-I{inc}" if f.startswith("-I") else f for f in flags]


def hipcc(args):
    subprocess.run([BN.HIPCC, *args], check=True)


def fresh(out: Path, *srcs: Path) -> bool:
    return out.exists() and all(out.stat().st_mtime >= s.stat().st_mtime for s in srcs)


def kernel_counts(asm: Path) -> str:
    body, inside = [], False
    for ln in asm.read_text().splitlines():
        if ln.startswith(KERNEL) and ": ;" in ln:
            inside = True
        elif inside and ln.startswith(".Lfunc_end"):
            break
        elif inside:
            body.append(re.sub(r"\.LBB\d+_\d+", "L", ln))
    keys = ("v_accvgpr_write", "v_accvgpr_read", "scratch_store", "scratch_load")
    return f"{len(body)} lines; " + ", ".join(f"{k} {sum(k in x for x in body)}" for k in keys), body


def main():
    assert FENCE[1] in BN.FLAGS, "build_native.py no longer carries the fence"
    OUT.mkdir(exist_ok=True)
    src = OUT / f"src_{REV}"
    if not (src / "yieldfactormodels.jl_amd" / "csrc").exists():
        src.mkdir(exist_ok=True)
        tar = subprocess.run(["git", "-C", str(ROOT), "archive", REV, "yieldfactormodels.jl_amd/csrc", "include"],
                             check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", str(src)], input=tar, check=True)
    csrc = src / "yieldfactormodels.jl_amd" / "csrc"
    flags = with_include(BN.FLAGS, src / "include")
    jobs = []
    objs = {"fenced": [], "unfenced": []}
    for s in sorted(csrc.glob("*.hip")):
        if s.stem == "yfm_kernels":  # the translation unit of the fixed-loading kernels: built both ways
            for tag, fl in (("fenced", flags), ("unfenced", unfenced(flags))):
                o = OUT / f"{REV}_{s.stem}_{tag}.o"
                objs[tag].append(o)
                jobs.append((o, [*fl, "-c", str(s), "-o", str(o)]))
        else:
            o = OUT / f"{REV}_{s.stem}.o"
            objs["fenced"].append(o)
            objs["unfenced"].append(o)
            jobs.append((o, [*flags, "-c", str(s), "-o", str(o)]))
    asm = {}
    for tag, fl, srcfile in (("fenced", flags, csrc / "yfm_kernels.hip"), ("unfenced", unfenced(flags), csrc / "yfm_kernels.hip"),
                             ("HEAD_fenced", BN.FLAGS, BN.CSRC / "yfm_kernels.hip"),
                             ("HEAD_unfenced", unfenced(BN.FLAGS), BN.CSRC / "yfm_kernels.hip")):
        a = OUT / f"kernels_{tag}.s"
        asm[tag] = a
        jobs.append((a, [*fl, "--offload-device-only", "-S", str(srcfile), "-o", str(a)]))
    # the fixed revision's outputs are reused once built; the HEAD assembly is rebuilt on every run (the in-tree
    # sources change, and the report below compares HEAD's fenced and unfenced code)
    todo = [args for o, args in jobs if not o.exists() or o.name.startswith("kernels_HEAD")]
    with ThreadPoolExecutor(max_workers=6) as ex:
        list(ex.map(hipcc, todo))
    for tag in ("fenced", "unfenced"):
        hipcc([f"--offload-arch={BN.ARCH}", "-shared", "-fPIC", *map(str, objs[tag]), "-o",
               str(OUT / f"libyfm_{REV}_{tag}.so")])
    subprocess.run(["g++", "-O2", "-std=c++17", str(HERE / "repro.cpp"), "-ldl", "-o", str(HERE / "repro")], check=True)
    rep = [f"two-function NP = 48 GNS5 kernel ({KERNEL}…), device assembly:"]
    bodies = {}
    for tag in asm:
        line, bodies[tag] = kernel_counts(asm[tag])
        rep.append(f"  {REV if not tag.startswith('HEAD') else 'HEAD'} {tag.replace('HEAD_', '')}: {line}")
    rep.append(f"  {REV}: fenced and unfenced code {'IDENTICAL' if bodies['fenced'] == bodies['unfenced'] else 'differ'}; "
               f"HEAD: {'IDENTICAL' if bodies['HEAD_fenced'] == bodies['HEAD_unfenced'] else 'differ'}")
    (OUT / "spill_report.txt").write_text("\n".join(rep) + "\n")
    print("\n".join(rep))


if __name__ == "__main__":
    main()
