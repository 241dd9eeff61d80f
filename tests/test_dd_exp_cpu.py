"""The certified kernels' dd_exp (yfm_dd.hpp: the table-driven dd_exp_core) against binary128 expq on the host:
tools/dd_exp_check.hip, compiled host-only, measures it and the Taylor-and-squarings version it replaced on 10⁶
arguments over five ranges and fails if the new one is worse than twice the old one + 8 u² anywhere (no GPU)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = Path("/opt/rocm/bin/hipcc")


def _quadmath_dirs():
    hdr = sorted(Path("/usr/lib/gcc").glob("*/*/include/quadmath.h"))
    lib = sorted(Path("/usr/lib/gcc").glob("*/*/libquadmath.so"))
    return (hdr[0].parent if hdr else None), (lib[0].parent if lib else None)


@pytest.mark.skipif(not HIPCC.exists() or None in _quadmath_dirs(), reason="hipcc or libquadmath missing")
def test_dd_exp_table_vs_binary128(tmp_path):
    inc, lib = _quadmath_dirs()
    exe = tmp_path / "dd_exp_check"
    subprocess.run([str(HIPCC), "-O2", "--offload-arch=gfx950", "--offload-host-only",
                    "-I", str(ROOT / "yieldfactormodels.jl_amd" / "csrc"), "-isystem", str(inc),
                    str(ROOT / "tools" / "dd_exp_check.hip"), f"-L{lib}", "-lquadmath", "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout
    # moderate arguments (the filters' λ and e^{−λm}): within a few u² of binary128
    first = r.stdout.splitlines()[1]
    assert float(first.split("table max ")[1].split(" u²")[0]) < 8.0, first
