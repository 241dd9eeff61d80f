"""CPU checks of the reference-format file I/O: DelimitedFiles-style CSV
writing/reading, Julia's round(x; digits), load_data/save_results paths and layouts.

The printed form of a Float64 follows Julia's `print` (shortest round-trip digits, scientific
outside [1e-4, 1e6)); the expected strings below are Julia's documented printing behaviour,
restated — parity unpinned (no Julia in this image).  Values always round-trip exactly."""
from __future__ import annotations

import numpy as np
import pytest

from yfm_amd import io as yio


@pytest.mark.parametrize("x,s", [
    (0.1, "0.1"), (1.0, "1.0"), (-2.0, "-2.0"), (100.0, "100.0"), (123456.0, "123456.0"),
    (0.0001, "0.0001"), (0.00012, "0.00012"), (1e-5, "1.0e-5"), (-2.5e-7, "-2.5e-7"), (1e6, "1.0e6"),
    (1234567.0, "1.234567e6"), (5e-324, "5.0e-324"), (1.7976931348623157e308, "1.7976931348623157e308"),
    (0.0, "0.0"), (-0.0, "-0.0"), (float("nan"), "NaN"), (float("inf"), "Inf"), (float("-inf"), "-Inf"),
    (3.141592653589793, "3.141592653589793"), (361.0, "361.0"), (0.30000000000000004, "0.30000000000000004"),
])
def test_julia_float_printing(x, s):
    assert yio.julia_float_str(x) == s


def test_writedlm_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    A = rng.standard_normal((7, 5)) * 10.0 ** rng.integers(-8, 9, size=(7, 5))
    A[0, 0], A[1, 1] = np.nan, -np.inf
    p = tmp_path / "a.csv"
    yio.writedlm(p, A)
    B = yio.readdlm(p)
    np.testing.assert_array_equal(A, B)
    yio.writedlm(p, np.arange(3.0))  # a vector: one value per line
    assert p.read_text() == "0.0\n1.0\n2.0\n"


def test_julia_round_ties_to_even():
    x = np.array([0.0025, 0.0125, 1.2345, -1.2355, 0.0005, 0.0015, np.nan])
    y = yio.julia_round(x, 3)
    np.testing.assert_array_equal(y[:6], np.rint(x[:6] * 1000) / 1000)
    assert y[4] == 0.0 and y[5] == 0.002  # ties to even
    assert np.isnan(y[6]) and yio.julia_round(1e300, 3) == 1e300  # non-finite x·10^d keeps x


def test_load_data_and_save_results(tmp_path):
    from yfm_amd import create_model, set_params_
    from yfm_amd import synthetic as S
    mats = S.maturities_30()
    Y = S.simulate_panel(0, 40)
    yio.writedlm(tmp_path / "thread_id__7__data.csv", Y)
    yio.writedlm(tmp_path / "thread_id__7__maturities.csv", mats)
    d, m = yio.load_data(str(tmp_path) + "/", "7")
    np.testing.assert_array_equal(d, Y)
    np.testing.assert_array_equal(m, mats)
    model, _ = create_model("1C", mats, 30, results_location=str(tmp_path) + "/res/")
    set_params_(model, S.theta0_constrained(0))
    res = dict(preds=np.ones((30, 40)), factors=np.zeros((3, 40)), states=np.full((1, 40), 2.0),
               factor_loadings_1=np.ones((30, 40)), factor_loadings_2=np.ones((30, 40)))
    yio.save_results(model, res, -12.5, "7", "insample")
    f = yio.readdlm(tmp_path / "res" / "1C__thread_id__7__factors_filtered_insample.csv")
    assert f.shape == (40, 4) and (f[:, 3] == 2.0).all()
    assert yio.readdlm(tmp_path / "res" / "1C__thread_id__7__fit_filtered_insample.csv").shape == (40, 30)
    assert (tmp_path / "res" / "1C__thread_id__7__loss.csv").read_text() == "-12.5\n"
    np.testing.assert_array_equal(yio.readdlm(tmp_path / "res" / "1C__thread_id__7__out_params.csv")[:, 0],
                                  S.theta0_constrained(0))
