"""Build an A/B variant of libyfm_hip.so: the in-tree objects (yieldfactormodels.jl_amd/build/, current) with
one or more translation units recompiled with extra flags, linked into tools/variants/<tag>.so.

    python tools/ab_build.py <tag> <tu>[,<tu>...] -DFOO=0 [-DBAR=1 ...]

(tu = a csrc file stem, e.g. yfm_tvl_dd).  Run tools/ab_run.sh on the GPU box to compare."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yieldfactormodels.jl_amd"))
import build_native as BN  # noqa: E402


def main():
    tag, tus, extra = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
    BN.build(verbose=False)  # the baseline objects must be current
    out = ROOT / "tools" / "variants"
    out.mkdir(exist_ok=True)
    objs = []
    for s in sorted(BN.CSRC.glob("*.hip")):
        o = BN.BUILD / (s.stem + ".o")
        if s.stem in tus:
            o = out / f"{tag}_{s.stem}.o"
            subprocess.run([BN.HIPCC, *BN.FLAGS, *extra, "-c", str(s), "-o", str(o)], check=True)
        objs.append(str(o))
    lib = out / f"{tag}.so"
    subprocess.run([BN.HIPCC, f"--offload-arch={BN.ARCH}", "-shared", "-fPIC", *objs, "-o", str(lib)], check=True)
    print(lib)


if __name__ == "__main__":
    main()
