"""Register and scratch budgets of the hot kernels, read from the gfx950 code objects inside the in-tree library
(no GPU needed).  The DNS kernel's speed rests on its register allocation (the MFMA A
fragments read from AGPRs, no scratch); a compiler or source change that makes it spill would cost several per
cent silently — this fails instead.  Budgets are the measured ones of the committed build."""
import re
import struct
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "yieldfactormodels.jl_amd" / "yfm_amd" / "libyfm_hip.so"
READELF = Path("/opt/rocm/lib/llvm/bin/llvm-readelf")

# kernel (demangled-name fragment of the mangled symbol) → max scratch bytes per lane
BUDGETS = {
    # config 2 / 4: DNS, NP = 30, loglik mode with the frozen-covariance steady state
    "fixedz_loglik_kernelILi30ELi3ELi1ELb0ELb1ELb0EE": 0,
    # the same with the full recursion (YFM_DNS_STEADY=0, the steady-vs-full gate)
    "fixedz_loglik_kernelILi30ELi3ELi1ELb0ELb0ELb0EE": 0,
    # config 5: GNS5, NP = 30, full recursion
    "fixedz_loglik_kernelILi30ELi5ELi2ELb0ELb0ELb0EE": 0,
    # config 5: the GNS5 initial state, two lanes per candidate (the per-lane kernel spills 540 B/lane)
    "fixedz_init_coop_kernelILi5ELi2ELi2E": 0,
    # config 3: certified TVλ at L = 4
    "tvl_dd_loglik_kernelILi4ELb0E": 0,
}


def _code_objects(data: bytes):
    """the gfx950 code objects of every clang offload bundle in the library"""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = data.find(magic)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        off = pos + 32
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tl].decode()
            off += tl
            if triple.endswith("gfx950"):
                yield data[pos + eo:pos + eo + es]
        pos = data.find(magic, pos + 1)


def _kernel_metadata(tmp_path):
    meta = {}
    for k, co in enumerate(_code_objects(LIB.read_bytes())):
        f = tmp_path / f"co{k}.elf"
        f.write_bytes(co)
        notes = subprocess.run([str(READELF), "--notes", str(f)], capture_output=True, text=True, check=True).stdout
        for entry in re.split(r"\n  - \.agpr_count:", notes)[1:]:
            name = re.search(r"\.name:\s+(\S+)", entry)
            if not name:
                continue
            fields = {key: int(v) for key, v in re.findall(
                r"\.(private_segment_fixed_size|vgpr_spill_count|vgpr_count|group_segment_fixed_size):\s+(\d+)", entry)}
            fields["agpr_count"] = int(entry.split("\n", 1)[0].strip())
            meta[name.group(1)] = fields
    return meta


@pytest.mark.skipif(not LIB.exists() or not READELF.exists(), reason="in-tree library or llvm-readelf missing")
def test_hot_kernels_within_register_budget(tmp_path):
    meta = _kernel_metadata(tmp_path)
    assert meta, "no gfx950 kernel metadata found in the library"
    for frag, max_scratch in BUDGETS.items():
        hits = [(n, m) for n, m in meta.items() if frag in n]
        assert hits, f"kernel {frag} not in the library"
        for name, m in hits:
            assert m["private_segment_fixed_size"] <= max_scratch, (name, m)
            # one wave per SIMD: the unified file holds 512 registers per lane
            assert m["vgpr_count"] <= 512, (name, m)


def test_bundle_parser_rejects_garbage():
    assert list(_code_objects(b"no bundle here")) == []
