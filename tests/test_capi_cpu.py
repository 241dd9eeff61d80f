"""CPU-side checks of the C ABI and the host mirror (no compute calls: no GPU here)."""
from __future__ import annotations

import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from oracle import kalman_oracle as O
from yfm_amd import _lib, params, synthetic as S
from yfm_amd.params import KIND_DNS, KIND_GNS, KIND_TVL


def header_symbols():
    txt = (ROOT / "include" / "yfm.h").read_text()
    return sorted(set(re.findall(r"\b(yfm_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 10
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                        check=True).stdout
    exported = set(re.findall(r" T (yfm_\w+)", nm))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    assert set(syms) == set(_lib.SIGNATURES), "ctypes binding and header disagree"
    for s in syms:
        getattr(lib, s)


def test_library_is_gfx950_code_object():
    data = _lib.LIB_PATH.read_bytes()  # the .hip_fatbin bundle names its offload target
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_abi_introspection():
    lib = _lib.load()
    assert lib.yfm_abi_version() == _lib.ABI_VERSION
    for kind in (KIND_DNS, KIND_TVL, KIND_GNS):
        assert lib.yfm_param_count(kind) == params.n_params(kind) == O.n_params(kind, params.state_dim(kind))
        assert lib.yfm_state_dim(kind) == params.state_dim(kind)
    assert lib.yfm_param_count(7) == -1
    assert params.n_params(KIND_DNS) == 20 and params.n_params(KIND_TVL) == 31


def test_create_without_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = _lib.load()
    assert not lib.yfm_create(0)
    assert b"device" in lib.yfm_last_error()


@pytest.mark.parametrize("kind", [KIND_DNS, KIND_TVL, KIND_GNS])
def test_host_transforms_match_oracle(kind):
    th = S.theta_batch(kind, 16, seed=7, bad_frac=0.0)
    codes = O.transform_codes(kind, params.state_dim(kind))
    assert list(codes) == list(params.transform_codes(kind))
    got = params.transform_params(kind, th)
    for b in range(th.shape[1]):
        np.testing.assert_array_equal(got[:, b], O.transform_params(codes, th[:, b]))
    np.testing.assert_allclose(params.untransform_params(kind, got), th, rtol=1e-12, atol=1e-13)


def test_create_model_mirror():
    from yfm_amd import DNSModel, TVLambdaDNSModel, create_model, get_params, set_params_
    mats = S.maturities_30()
    m, std = create_model("0", mats, 30, 3)
    assert isinstance(m, DNSModel) and std == "1C"
    m2, std2 = create_model("TVλ", mats, 30, 3)
    assert isinstance(m2, TVLambdaDNSModel) and std2 == "TVλ" and m2.base.M == 4
    with pytest.raises(ValueError):
        create_model("NNS", mats, 30, 3)
    set_params_(m, S.theta0_constrained(KIND_DNS))
    np.testing.assert_array_equal(get_params(m), S.theta0_constrained(KIND_DNS))
    with pytest.raises(ValueError):
        set_params_(m, np.zeros(5))


def test_build_keeps_agpr_spill_fence():
    """DESIGN.md §5 / VERDICT r4 item 7: the library must be built with `-mllvm -amdgpu-spill-vgpr-to-agpr=0`
    (ROCm 7.2 miscompiled the VGPR→AGPR spill path of the spilling GNS5 NP = 48 kernel;
    tools/agpr_spill_repro/ reproduces it).  Dropping the fence from build_native.py fails here, loudly,
    in the default CPU suite — and the stamp of the objects actually linked must carry it too."""
    import build_native as BN
    i = BN.FLAGS.index("-amdgpu-spill-vgpr-to-agpr=0")
    assert BN.FLAGS[i - 1] == "-mllvm", BN.FLAGS
    if BN.STAMP.exists():  # the library in the tree was linked from objects built with the fence
        assert "-amdgpu-spill-vgpr-to-agpr=0" in BN.STAMP.read_text().split("\n")
