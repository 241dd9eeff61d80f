"""CPU test of the estimation driver's host logic (yfm_nm.hpp): the
Nelder–Mead chain state machine and the speculation tree of later iterations, driven by a host
objective through the same prepare → evaluate → absorb rounds yfm_estimate runs.

* Every tree budget (1 = one iteration per round, 7, 16 = the default, 32) gives bitwise the same
  chains and evaluation counts — speculation only changes how many iterations a round covers.
* The chains equal oracle/optim_nm.py's estimate_steps! (Optim.jl NelderMead restated, identity
  transforms) bit for bit, including the ×0.95 rescaling of a start whose objective is +Inf
  (optimization.jl:173-184).
"""
from __future__ import annotations

import math
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from oracle import optim_nm as NM

R, N, ITER, MGI = 6, 20, 120, 3


def py_objective(r):
    def f(x):
        if x[0] > 5.0:
            return math.inf
        s = 0.0
        for i in range(N):
            d = x[i] - 0.1 * (i % 5) - 0.01 * r
            s = s + (1.0 + 0.25 * (i % 3)) * d * d
        for i in range(N - 1):
            s = s + 0.05 * x[i] * x[i + 1]
        return s
    return f


def start(r):
    p = np.array([(0.2 * ((i * 7 + r * 3) % 11)) / 11.0 - 0.1 for i in range(N)])
    if r == 0:
        p[0] = 6.0
    return p


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = tmp_path_factory.mktemp("nm") / "nm_tree_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wno-unknown-pragmas",
                    str(ROOT / "tests" / "nm_tree_check.cpp"), "-o", str(exe)], check=True)
    return exe


def run(exe, budget):
    out = subprocess.run([str(exe), str(R), str(N), str(budget), str(ITER), str(MGI)], check=True,
                         capture_output=True, text=True).stdout.split("\n")
    rounds = int(out[0].split()[1])
    chains = []
    for line in out[1:1 + R]:
        f = line.split()
        chains.append((int(f[1]), int(f[2]), float.fromhex(f[3]), [float.fromhex(v) for v in f[4:]]))
    return rounds, chains


def test_tree_budgets_bitwise_neutral(harness):
    r1, base = run(harness, 1)
    for budget in (7, 16, 32):
        rb, got = run(harness, budget)
        assert got == base, budget
        assert rb < r1  # speculation covers several iterations per round


def test_chains_equal_oracle(harness):
    _, got = run(harness, 16)
    for r in range(R):
        ref = NM.estimate_steps(py_objective(r), start(r), transform=lambda x: x, untransform=lambda x: x,
                                max_group_iters=MGI, iterations=ITER)
        status, used, ll, p = got[r]
        assert status == ref.status == 0
        assert ll == ref.ll and np.array_equal(np.array(p), ref.p), r
        # (n_evals counts the points a chain consumes, four per iteration as the device rounds
        # evaluate them, not Optim's one-or-two objective calls per iteration)
        assert used > ref.f_calls
