"""GPU parity: libyfm_hip.so (through the C ABI) vs the oracle / committed golden fixtures.

Tolerance (north star, BASELINE.json): 1e-9 relative on loglik and on the filtered
states, FP64; -Inf / NaN patterns must match exactly.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import GOLDEN_NAMES, ROOT, load_golden
from yfm_amd import KIND_DNS, KIND_GNS, KIND_TVL, _lib
from yfm_amd import synthetic as S
from yfm_amd.params import n_params

pytestmark = pytest.mark.gpu

REL = 1e-9


def assert_ll_close(got, ref, rel=REL):
    got, ref = np.asarray(got), np.asarray(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref)), (got, ref)
    assert np.array_equal(np.isneginf(got), np.isneginf(ref)), (got, ref)
    assert not np.isposinf(got).any()
    fin = np.isfinite(ref)
    if fin.any():
        err = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)
        # loglik exactly 0.0 (T_use ≤ 2) must be exact
        assert np.all((ref[fin] != 0.0) | (got[fin] == 0.0))
        assert err.max() <= rel, (err.max(), np.argmax(err))


def assert_parity(got, oracle, truth=None, rel=REL):
    """North-star parity: within `rel` (1e-9) of the FP64 oracle — or, where the two differ by
    more, at least as close to exact arithmetic as the oracle is (factor 1): |gpu − truth| ≤
    |oracle − truth|, truth = a 40-digit or binary128 evaluation of the same recursion
    (oracle/kalman_mp.py, oracle/yfm_truth.c).  NaN / −Inf patterns must match exactly."""
    got, oracle = np.asarray(got, dtype=np.float64), np.asarray(oracle, dtype=np.float64)
    if truth is None:
        return assert_ll_close(got, oracle, rel)
    truth = np.asarray(truth, dtype=np.float64)
    assert np.array_equal(np.isnan(got), np.isnan(oracle)) and np.array_equal(np.isneginf(got), np.isneginf(oracle))
    fin = np.isfinite(oracle)
    den_t = np.maximum(np.abs(truth[fin]), 1e-300)  # loglik exactly 0.0 (T_use ≤ 2) must be exact
    e_or = np.abs(oracle[fin] - truth[fin]) / den_t
    e_go = np.abs(got[fin] - oracle[fin]) / np.maximum(np.abs(oracle[fin]), 1e-300)
    e_gt = np.abs(got[fin] - truth[fin]) / den_t
    ok = (e_go <= rel) | (e_gt <= e_or)
    assert ok.all(), (e_go[~ok], e_gt[~ok], e_or[~ok])
    return parity_table(got, oracle, truth, rel)


def parity_table(got, oracle, truth, rel=REL) -> dict:
    """(within 1e-9 of the oracle, adjudicated: further but at least as close to truth, failing)."""
    fin = np.isfinite(oracle) & np.isfinite(got)
    den = np.maximum(np.abs(truth[fin]), 1e-300)
    e_go = np.abs(got[fin] - oracle[fin]) / np.maximum(np.abs(oracle[fin]), 1e-300)
    e_gt = np.abs(got[fin] - truth[fin]) / den
    e_or = np.abs(oracle[fin] - truth[fin]) / den
    within = e_go <= rel
    adj = ~within & (e_gt <= e_or)
    return {"n": int(fin.sum()), "within_1e-9": int(within.sum()), "adjudicated": int(adj.sum()),
            "failing": int((~within & ~adj).sum()), "gpu_vs_truth_max_rel": float(e_gt.max()) if e_gt.size else 0.0,
            "oracle_vs_truth_max_rel": float(e_or.max()) if e_or.size else 0.0}


def supported(kind):
    return kind in (KIND_DNS, KIND_GNS, KIND_TVL)


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_golden_loglik(engine, name):
    g = load_golden(name)
    kind = int(g["kind"])
    if not supported(kind):
        pytest.skip("TVλ kernel not built yet")
    engine.set_panel(g["Y"], g["maturities"])
    got = engine.loglik(kind, g["Theta"], space=int(g["space"]), T_use=g.get("T_use"))
    if "ll_truth" in g:
        k = len(g["ll_truth"])
        assert_parity(got[:k], g["loglik"][:k], g["ll_truth"])
        assert_ll_close(got[k:], g["loglik"][k:])
    else:
        assert_ll_close(got, g["loglik"])


@pytest.mark.parametrize("name", [n for n in GOLDEN_NAMES if "beta_traj" in load_golden(n)])
def test_golden_states(engine, name):
    """Filtered states a_{t+1|t}, P_{t+1|t} after every filter! call.

    Two checks per trajectory, normwise per array (scale = max |truth|):
      * factor 1: within 1e-9 of the FP64 oracle, or — where the reference's dense FP64
        arithmetic is itself further than that from exact arithmetic (the I − KZ
        cancellation) — at least as close to the ground truth as the oracle;
      * vs the 40-digit ground truth (oracle/kalman_mp.py): within 1e-10.
    """
    g = load_golden(name)
    kind = int(g["kind"])
    if not supported(kind):
        pytest.skip("TVλ kernel not built yet")
    engine.set_panel(g["Y"], g["maturities"])
    nt = g["beta_traj"].shape[-1]
    ll, beta, P = engine.filter_states(kind, g["Theta"][:, :nt], space=int(g["space"]))
    assert_parity(ll, g["loglik"][:nt], g["ll_truth"])
    for b in range(nt):
        if not np.isfinite(g["loglik"][b]):
            continue
        for got, ora, tru in ((beta[..., b], g["beta_traj"][..., b], g["beta_truth"][..., b]),
                              (P[..., b], g["P_traj"][..., b], g["P_truth"][..., b])):
            scale = np.abs(tru).max()
            e_ot = np.abs(ora - tru).max() / scale
            e_go = np.abs(got - ora).max() / scale
            e_gt = np.abs(got - tru).max() / scale
            assert e_go <= REL or e_gt <= e_ot, (name, b, e_go, e_gt, e_ot)
            assert e_gt <= 1e-10


@pytest.fixture(scope="module")
def headline():
    Y = S.simulate_panel(KIND_DNS, 600)
    return Y, S.maturities_30()


def test_headline_shape_vs_c_oracle(engine, headline):
    """N = 30, T = 600 (config 1/2 shape), 256 candidates incl. 5% non-stationary Φ, vs the C oracle,
    adjudicated by the binary128 truth (oracle/yfm_truth.c) where the oracle is off."""
    from oracle.truth import loglik_truth
    import ctypes
    Y, mats = headline
    Th = S.theta_batch(KIND_DNS, 256, seed=99, bad_frac=0.05)
    engine.set_panel(Y, mats)
    got = engine.loglik(KIND_DNS, Th)
    lib = ctypes.CDLL(str(ROOT / "oracle" / "libyfm_oracle.so"))
    D = ctypes.POINTER(ctypes.c_double)
    ref = np.empty(256)
    Yf = np.asfortranarray(Y)
    lib.yfm_oracle_loglik(KIND_DNS, 0, Yf.ctypes.data_as(D), 30, 600, mats.ctypes.data_as(D),
                          Th.ctypes.data_as(D), 20, 256, None, ref.ctypes.data_as(D), 0)
    assert_parity(got, ref, loglik_truth(KIND_DNS, Y, mats, Th))


def test_full_batch_properties(engine, headline):
    """B = 65,536 (config 2): results are independent of batch position and size, deterministic, and the
    flag counters match the NaN/-Inf outputs."""
    Y, mats = headline
    engine.set_panel(Y, mats)
    Th = S.theta_batch(KIND_DNS, 65536)
    a = engine.loglik(KIND_DNS, Th)
    n_throw, n_neginf = engine.last_flags()
    assert n_throw == np.isnan(a).sum() and n_neginf == np.isneginf(a).sum()
    b = engine.loglik(KIND_DNS, Th)
    np.testing.assert_array_equal(a, b)  # bit-deterministic
    perm = np.random.default_rng(1).permutation(65536)[:1000]
    c = engine.loglik(KIND_DNS, np.asfortranarray(Th[:, perm]))
    np.testing.assert_array_equal(c, a[perm])  # position/size independent
    assert np.isfinite(a).mean() > 0.95


def test_constrained_equals_unconstrained(engine, headline):
    from yfm_amd.params import transform_params
    Y, mats = headline
    engine.set_panel(Y[:, :200], mats)
    Th = S.theta_batch(KIND_DNS, 64, seed=4, bad_frac=0.0)
    a = engine.loglik(KIND_DNS, Th, space=0)
    b = engine.loglik(KIND_DNS, transform_params(KIND_DNS, Th), space=1)
    assert_ll_close(a, b, rel=1e-11)  # host numpy exp vs device exp: 1-ulp differences in θ_c


def test_device_pointer_api_matches_host_api(engine, headline):
    import torch
    Y, mats = headline
    engine.set_panel(Y, mats)
    Th = S.theta_batch(KIND_DNS, 4096, seed=8)
    ref = engine.loglik(KIND_DNS, Th)
    dth = torch.from_numpy(np.ascontiguousarray(Th.T)).cuda()  # (B, P) C-order == P×B column-major
    out = torch.empty(4096, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    engine.loglik_device(KIND_DNS, dth.data_ptr(), 20, 4096, out.data_ptr(), space=0, stream=s.cuda_stream)
    s.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("kind", [KIND_DNS, KIND_GNS])
def test_pipelined_host_batch_matches_device_launch(engine, headline, kind):
    """B ≥ 2×131,072: yfm_loglik_batch uploads θ in chunks on a copy stream while earlier chunks
    run; the logliks equal one device-pointer launch bit for bit, with ragged T_use windows, and
    the flag counters cover every chunk."""
    import torch
    Y, mats = headline
    engine.set_panel(Y[:, :120], mats)
    B = 300_001  # three chunks, the last one ragged
    P = n_params(kind)
    Th = S.theta_batch(kind, B, seed=31, bad_frac=0.05)
    tu = np.random.default_rng(5).integers(2, 121, B).astype(np.int32)
    got = engine.loglik(kind, Th, T_use=tu)
    n_throw, n_neginf = engine.last_flags()
    assert n_throw == np.isnan(got).sum() and n_neginf == np.isneginf(got).sum()
    dth = torch.from_numpy(np.ascontiguousarray(Th.T)).cuda()
    dtu = torch.from_numpy(tu).cuda()
    out = torch.empty(B, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    engine.loglik_device(kind, dth.data_ptr(), P, B, out.data_ptr(), space=0, d_T_use=dtu.data_ptr(),
                         stream=s.cuda_stream)
    s.synchronize()
    np.testing.assert_array_equal(got, out.cpu().numpy())


def test_windows_share_prefix(engine, headline):
    """T_use windows: candidate with T_use = τ equals a full evaluation on data[:, :τ]."""
    Y, mats = headline
    Th = S.theta_batch(KIND_DNS, 8, seed=21, bad_frac=0.0)
    Th = np.asfortranarray(np.repeat(Th, 3, axis=1))
    tu = np.array([361, 480, 600] * 8, dtype=np.int32)
    engine.set_panel(Y, mats)
    got = engine.loglik(KIND_DNS, Th, T_use=tu)
    for tau in (361, 480, 600):
        engine.set_panel(Y[:, :tau], mats)
        ref = engine.loglik(KIND_DNS, Th[:, tu == tau])
        np.testing.assert_array_equal(got[tu == tau], ref)


def test_edge_sizes(engine, headline):
    Y, mats = headline
    engine.set_panel(Y[:, :1], mats)
    np.testing.assert_array_equal(engine.loglik(KIND_DNS, S.theta_batch(KIND_DNS, 3, bad_frac=0.0)), 0.0)
    engine.set_panel(Y[:, :50], mats)
    assert engine.loglik(KIND_DNS, np.zeros((20, 0))).shape == (0,)
    with pytest.raises(ValueError):
        engine.loglik(KIND_DNS, np.zeros((19, 4)))  # wrong P (host check)
    with pytest.raises(_lib.YFMError):
        engine.loglik(KIND_DNS, np.zeros((20, 2)), T_use=np.array([0, 5]))  # C-ABI check
    lib = engine.lib
    th = np.zeros((19, 2))
    out = np.zeros(2)
    assert lib.yfm_loglik_batch(engine.ctx, 0, 0, _lib.dptr(th), 19, 2, None, _lib.dptr(out)) == -1
    assert b"P = 19" in lib.yfm_last_error()


def test_model_api_mirror(engine, headline):
    """create_model / set_params_ / get_loss / compute_loss mirror the reference's call sequence."""
    from oracle import kalman_oracle as O
    from yfm_amd import compute_loss, compute_loss_batch, create_model, get_loss, set_params_
    Y, mats = headline
    Y = Y[:, :150]
    model, _ = create_model("1C", mats, 30, 3)
    th = S.theta0(KIND_DNS)
    ref = O.loglik(KIND_DNS, mats, 3, Y, th)
    assert abs(-compute_loss(model, Y, th) - ref) <= REL * abs(ref)
    set_params_(model, S.theta0_constrained(KIND_DNS))
    assert abs(get_loss(model, Y) - ref) <= 1e-9 * abs(ref)
    Th = S.theta_batch(KIND_DNS, 16, seed=2, bad_frac=0.0)
    cl = compute_loss_batch(model, Y, Th)
    assert abs(-cl[0] - O.loglik(KIND_DNS, mats, 3, Y, Th[:, 0])) <= REL * abs(cl[0])


def test_pinned_host_buffers(engine, headline):
    """yfm_alloc_host / yfm_free_host: θ and logliks in page-locked memory give the same bits."""
    Y, mats = headline
    engine.set_panel(Y, mats)
    Th = S.theta_batch(KIND_DNS, 5000, seed=17)
    ref = engine.loglik(KIND_DNS, Th)
    th_pin = engine.host_array(Th.shape)
    th_pin[...] = Th
    out = engine.host_array((5000,))
    got = engine.loglik(KIND_DNS, th_pin, out=out)
    assert got is out
    np.testing.assert_array_equal(out, ref)
    del th_pin, out, got


@pytest.mark.parametrize("kind", [KIND_DNS, KIND_GNS])
@pytest.mark.parametrize("N", [5, 12, 20, 30, 31, 40, 60])
def test_every_panel_width_instantiation(engine, kind, N):
    """Every padded width the per-lane kernel is instantiated for (NP = 8, 16, 24, 30, 32, 48, 64;
    MFMA Z'ỹ up to 32, VALU dot products above) for both fixed-loading models vs the dense oracle,
    adjudicated by the binary128 truth.  (Round 3: a register-spilling instantiation (GNS5, NP = 48)
    computed wrong values with the update split into two functions — this pins every width.)"""
    from oracle.truth import loglik_oracle, loglik_truth
    rng = np.random.default_rng(N + 100 * kind)
    mats = np.sort(rng.choice(np.arange(3, 361), N, replace=False)).astype(np.float64)
    Y = S.simulate_panel(kind, 80, maturities=mats)
    Th = S.theta_batch(kind, 256, seed=N, bad_frac=0.02, scale=0.05)
    engine.set_panel(Y, mats)
    got = engine.loglik(kind, Th)
    assert_parity(got, loglik_oracle(kind, Y, mats, Th), loglik_truth(kind, Y, mats, Th))
