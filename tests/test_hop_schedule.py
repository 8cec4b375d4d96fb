"""CPU: the LightGCN hop schedules (functional.lightgcn_hop_schedule) simulated with the
epilogue semantics of include/gnnrec.h (ACC_INIT / ACC_ADD / ACC_X / ACC_DIV / NO_Y) over the
oracle's SpMM: the deferred (column-ordered kernel) schedule gives the eager schedule's bits
for every K, never gathers from rows it writes, and moves fewer epilogue rows."""
import numpy as np
import pytest

import oracle
from conftest import golden_csr

from src.ops import functional as F
from src.ops._lib import EPI_ACC_ADD, EPI_ACC_DIV, EPI_ACC_INIT, EPI_ACC_X, EPI_NO_Y


def run(sched, rp, col, val, x0, K):
    bufs = {"x0": x0, "acc": np.full_like(x0, np.nan), "a": None, "b": None}
    moved = 0
    for xn, yn, epi in sched:
        x = bufs[xn]
        writes_acc = bool(epi & (EPI_ACC_INIT | EPI_ACC_ADD))
        assert not (writes_acc and xn == "acc"), "a hop gathers from the rows it writes"
        assert xn != yn
        y = oracle.spmm(rp, col, val, x)
        if not (epi & EPI_NO_Y):
            assert yn is not None
            bufs[yn] = y.copy()
            moved += 1
        if writes_acc:
            terms = []
            if epi & EPI_ACC_INIT:
                terms.append(x0)
            if epi & EPI_ACC_ADD:
                terms.append(bufs["acc"])
            if epi & EPI_ACC_X:
                terms.append(x)
            b = terms[0]
            for t in terms[1:]:
                b = b + t
            b = b + y
            if epi & EPI_ACC_DIV:
                b = b / np.float32(K + 1)
            bufs["acc"] = b
            moved += len(terms) + 1
    return bufs["acc"], moved


@pytest.mark.parametrize("K", [1, 2, 3, 4, 5])
def test_deferred_schedule_same_bits(K):
    rp, col, val, _, _ = golden_csr("g_small")
    n = rp.shape[0] - 1
    x0 = np.random.default_rng(K).standard_normal((n, 64)).astype(np.float32) * np.float32(0.1)
    eager, m_e = run(F.lightgcn_hop_schedule(K, deferred=False), rp, col, val, x0, K)
    deferred, m_d = run(F.lightgcn_hop_schedule(K, deferred=True), rp, col, val, x0, K)
    np.testing.assert_array_equal(eager.view(np.uint32), deferred.view(np.uint32))
    # the reference's own form: torch.stack(all).mean(0) (lightgcn.py:94-95) as sequential adds
    layers, x = [x0], x0
    for _ in range(K):
        x = oracle.spmm(rp, col, val, x)
        layers.append(x)
    want = layers[0]
    for t in layers[1:]:
        want = want + t
    want = want / np.float32(K + 1)
    np.testing.assert_array_equal(eager.view(np.uint32), want.view(np.uint32))
    assert m_e == {1: 2, 2: 5, 3: 8, 4: 11, 5: 14}[K]
    assert m_d == {1: 2, 2: 4, 3: 6, 4: 9, 5: 12}[K]
