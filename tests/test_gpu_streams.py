"""Stream ordering of one context's launches (include/yfm.h, yfm_capi.hip: launch / settle_foreign_launch).

A context's device scratch and counters serve one launch at a time.  Launches on one stream are ordered by
the stream; after an asynchronous launch on a caller's stream, a synchronous entry point (yfm_loglik_batch
on the context's own stream, yfm_set_panel) waits for the device before it touches the shared buffers; a
caller that moves between its own streams orders them itself.  These tests run those transitions back to
back, without host synchronisation where the contract says none is needed, and compare every result with
the same batch evaluated alone; the per-launch counters (yfm_last_batch_flags) must belong to the launch
they are read after.  Reference: filter.jl:182-209 (get_loss, whose values are compared)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from yfm_amd import KIND_DNS
from yfm_amd import synthetic as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def panel():
    return S.simulate_panel(KIND_DNS, 600), S.maturities_30()


def test_device_launch_then_synchronous_call(engine, panel):
    Y, mats = panel
    engine.set_panel(Y, mats)
    Th = S.theta_batch(KIND_DNS, 65536, seed=21, bad_frac=0.02)
    Th2 = S.theta_batch(KIND_DNS, 4096, seed=22, bad_frac=0.05)
    ref = engine.loglik(KIND_DNS, Th)
    ref2 = engine.loglik(KIND_DNS, Th2)
    d_th = torch.from_numpy(np.ascontiguousarray(Th.T)).cuda()  # column b of Θ contiguous (P×B, F-order)
    d_out = torch.empty(Th.shape[1], dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        engine.loglik_device(KIND_DNS, d_th.data_ptr(), Th.shape[0], Th.shape[1], d_out.data_ptr(),
                             stream=s.cuda_stream)
    # no synchronisation: the synchronous call on the context's own stream must wait for the device
    got2 = engine.loglik(KIND_DNS, Th2)
    s.synchronize()
    np.testing.assert_array_equal(got2, ref2)
    np.testing.assert_array_equal(d_out.cpu().numpy(), ref)


def test_caller_stream_switch_with_caller_ordering(engine, panel):
    Y, mats = panel
    engine.set_panel(Y, mats)
    Th = S.theta_batch(KIND_DNS, 8192, seed=23, bad_frac=0.05)
    ref = engine.loglik(KIND_DNS, Th)
    n_neg = int((np.isneginf(ref)).sum())
    d_th = torch.from_numpy(np.ascontiguousarray(Th.T)).cuda()
    outs = [torch.empty(Th.shape[1], dtype=torch.float64, device="cuda") for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    ev = None
    for s, o in zip(streams, outs):
        if ev is not None:
            s.wait_event(ev)  # the caller orders its stream switch (include/yfm.h)
        engine.loglik_device(KIND_DNS, d_th.data_ptr(), Th.shape[0], Th.shape[1], o.data_ptr(), stream=s.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(s)
    streams[-1].synchronize()
    for o in outs:
        np.testing.assert_array_equal(o.cpu().numpy(), ref)
    # the counters read after the last launch are that launch's (a fresh bank on every stream change)
    flags = engine.last_flags()
    assert flags[1] == n_neg, (flags, n_neg)


def test_set_panel_after_device_launch(engine, panel):
    Y, mats = panel
    engine.set_panel(Y, mats)
    Th = S.theta_batch(KIND_DNS, 65536, seed=24)
    ref = engine.loglik(KIND_DNS, Th)
    d_th = torch.from_numpy(np.ascontiguousarray(Th.T)).cuda()
    d_out = torch.empty(Th.shape[1], dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    engine.loglik_device(KIND_DNS, d_th.data_ptr(), Th.shape[0], Th.shape[1], d_out.data_ptr(), stream=s.cuda_stream)
    # a new panel while that launch may still read the old one: set_panel waits for the device first
    Y2 = S.simulate_panel(KIND_DNS, 600, seed=99)
    engine.set_panel(Y2, mats)
    s.synchronize()
    np.testing.assert_array_equal(d_out.cpu().numpy(), ref)
    engine.set_panel(Y, mats)
