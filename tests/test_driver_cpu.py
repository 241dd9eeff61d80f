"""CPU checks of the one-call driver's host logic (yfm_amd.driver, mirroring src/YieldFactorModels.jl:
88-155, :221-347): data paths, parameter groups, load_initial_parameters! (read, or write a seeded random
start), and load_static_parameters! (TVλ seeded from a fitted DNS; DNS unchanged).  No compute call."""
from __future__ import annotations

import numpy as np

from yfm_amd import create_model
from yfm_amd import driver as Dv
from yfm_amd import io as yio
from yfm_amd import synthetic as S


def test_setup_data_paths():
    assert Dv.setup_data_paths("1C", False, "/s/", "3") == ("/s/YieldFactorModels.jl/data/",
                                                          "/s/YieldFactorModels.jl/results/thread_id__3/")
    assert Dv.setup_data_paths("1C", True, "", "3") == ("YieldFactorModels.jl/data_simulation/",
                                                      "YieldFactorModels.jl/results_simulation/thread_id__3/")


def test_param_groups_default_all_one():
    m, _ = create_model("1C", S.maturities_30(), 30)
    assert Dv.get_param_groups(m, []) == ["1"] * 20
    g = ["1"] * 19 + ["2"]
    assert Dv.get_param_groups(m, g) == g


def test_load_initial_parameters_reads_or_writes(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    m, _ = create_model("0", S.maturities_30(), 30)  # init folder uses the code as given ("0")
    a = Dv.load_initial_parameters_(m, "1C", rng=np.random.default_rng(43))
    f = tmp_path / "YieldFactorModels.jl/initializations/0/init_params_1C.csv"
    assert a.shape == (20, 1) and f.exists() and ((a >= 0) & (a < 1)).all()
    np.testing.assert_array_equal(yio.readdlm(f), a)
    th = np.column_stack([S.theta0_constrained(0), S.theta0_constrained(0) * 0.9])
    yio.writedlm(f, th)
    np.testing.assert_array_equal(Dv.load_initial_parameters_(m, "1C"), th)
    sim = tmp_path / "YieldFactorModels.jl/initializations/0/init_params_1C_simulation.csv"
    yio.writedlm(sim, th[:, :1] * 2)
    np.testing.assert_array_equal(Dv.load_initial_parameters_(m, "1C", simulation=True), th[:, :1] * 2)


def test_static_parameters_tvl_from_dns(tmp_path):
    loc = str(tmp_path) + "/"
    dns = S.theta0_constrained(0)  # [γ, σ², U(6), δ(3), Φ(9 row-major)]
    (tmp_path / "1C").mkdir()
    yio.writedlm(tmp_path / "1C" / "1C__thread_id__5__out_params.csv", dns)
    tvl, _ = create_model("TVλ", S.maturities_30(), 30)
    p0 = np.arange(31, dtype=np.float64) + 100.0
    p = Dv.load_static_parameters_(tvl, "TVλ", loc, "5", p0)
    exp = p0.copy()  # paramoperations.jl:78-90, 1-based → 0-based
    exp[0] = dns[1]
    exp[1:7] = dns[2:8]
    exp[11:14] = dns[8:11]
    exp[15:18], exp[19:22], exp[23:26] = dns[11:14], dns[14:17], dns[17:20]
    np.testing.assert_array_equal(p, exp)
    # DNS: no mapping in the reference (its try ends in the catch), with or without the file
    (tmp_path / "DNS").mkdir()
    yio.writedlm(tmp_path / "DNS" / "DNS__thread_id__5__out_params.csv", dns)
    m, _ = create_model("1C", S.maturities_30(), 30)
    q = np.arange(20.0)
    np.testing.assert_array_equal(Dv.load_static_parameters_(m, "1C", loc, "5", q), q)
    np.testing.assert_array_equal(Dv.load_static_parameters_(tvl, "TVλ", loc, "6", p0), p0)  # no file
