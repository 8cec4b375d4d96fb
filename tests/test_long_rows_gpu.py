"""Config 2's ML-1M-shaped graph on the GPU against the reference ITSELF
(tests/golden/lightgcn_ml1m_K3_d64.npz, made by the reference's graph_builder + LightGCN):
rows of up to 5 857 neighbours, 343 rows above the heavy-row threshold. Every kernel that can
run a LightGCN hop — the row-parallel CSR kernel alone, with the workgroup-per-row heavy
kernel at two thresholds, the column-ordered tiled kernel forced onto this small operand at
three block sizes, the fused K-hop launch, and the model class — must reproduce every layer
bit for bit (SHA-256 of the fp32 bytes), i.e. torch.sparse.mm's per-row chain order on long
rows (lightgcn.py:76-95)."""
import numpy as np
import pytest
import torch

from conftest import long_rows_case, sha256

from src.models import LightGCN
from src.ops import CsrGraph, functional as F
from src.ops._lib import EPI_ACC_ADD, EPI_ACC_DIV, EPI_ACC_INIT, EPI_NO_Y

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def case(cuda):
    f, u, i, nu, ni, x0 = long_rows_case()
    g = CsrGraph.from_interactions(u, i, nu, ni)
    assert [sha256(g.row_ptr.numpy()), sha256(g.col.numpy()), sha256(g.val.numpy())] == \
        list(f["operand_sha256"])
    return f, g.to(cuda), x0.to(cuda), nu, ni


def check_layers(f, hops, out=None):
    for k, y in enumerate(hops):
        got = y.detach().cpu().numpy()
        np.testing.assert_array_equal(got[f["heavy_rows"]].view(np.uint32),
                                      f["layers_heavy"][k].view(np.uint32), err_msg=f"hop {k + 1}")
        assert sha256(got) == f["layers_sha256"][k + 1], f"hop {k + 1} differs from the reference"
    if out is not None:
        o = out.detach().cpu().numpy()
        np.testing.assert_array_equal(o, np.concatenate([f["user_out"], f["item_out"]]))
        assert sha256(o) == f["out_sha256"]


def test_device_builder_matches_reference_operand(cuda):
    f, u, i, nu, ni, _ = long_rows_case()
    g = CsrGraph.from_interactions_device(u, i, nu, ni, device=cuda)
    assert [sha256(g.row_ptr.cpu().numpy()), sha256(g.col.cpu().numpy()),
            sha256(g.val.cpu().numpy())] == list(f["operand_sha256"])


@pytest.mark.parametrize("heavy", [0, 256, 16])
def test_csr_hops_bit_exact(case, heavy):
    """heavy=0: every row (5 857 neighbours included) in the row-parallel kernel; 256: the
    shipped split; 16: thousands of rows through the workgroup-per-row kernel."""
    f, g, x0, _, _ = case
    hops, x = [], x0
    for _ in range(3):
        y = torch.empty_like(x0)
        F.spmm_into(g, x, y, heavy_threshold=heavy)
        hops.append(y)
        x = y
    check_layers(f, hops)


@pytest.mark.parametrize("rows_per_block", [1279, 600, 97, 8])
def test_tiled_hops_bit_exact(case, rows_per_block):
    """The column-ordered kernel (forced: the operand is below TILED_MIN_ROWS) with the layer
    mean fused as in the headline path."""
    f, g, x0, _, _ = case
    plan = g.tiled_plan(rows_per_block=rows_per_block)
    acc = torch.empty_like(x0)
    hops, x = [], x0
    for k in range(1, 4):
        y = torch.empty_like(x0)
        epi = (EPI_ACC_INIT if k == 1 else EPI_ACC_ADD) | (EPI_ACC_DIV if k == 3 else 0)
        F.spmm_tiled_into(g, x, y, plan, epi=epi, self_rows=x0, acc=acc, acc_div=4.0)
        hops.append(y)
        x = y
    check_layers(f, hops, acc)
    # the headline form (last hop without y) gives the same mean
    acc2 = torch.empty_like(x0)
    x = x0
    for k in range(1, 4):
        last = k == 3
        y = None if last else torch.empty_like(x0)
        epi = (EPI_ACC_INIT if k == 1 else EPI_ACC_ADD) | ((EPI_ACC_DIV | EPI_NO_Y) if last else 0)
        F.spmm_tiled_into(g, x, y, plan, epi=epi, self_rows=x0, acc=acc2, acc_div=4.0)
        x = y
    assert torch.equal(acc, acc2)


def test_fused_propagation_bit_exact(case):
    f, g, x0, _, _ = case
    out, layers = F.lightgcn_forward(g, x0, 3, return_layers=True)
    check_layers(f, list(layers), out)
    out2, _ = F.lightgcn_forward(g, x0, 3)
    assert torch.equal(out, out2)


def test_model_class_bit_exact(case, cuda):
    f, g, _, nu, ni = case
    torch.manual_seed(int(f["seed"]))
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1).to(cuda).eval()
    with torch.no_grad():
        u, i = m(g)
        layers = m.get_layer_embeddings(g)
    check_layers(f, layers[1:], torch.cat([u, i]))
    # the reference's own operand form (uncoalesced torch COO moved to the device)
    with torch.no_grad():
        u2, i2 = m(g.to_torch_sparse_coo())
    assert torch.equal(u, u2) and torch.equal(i, i2)


@pytest.mark.parametrize("rows_per_block", [1279, 97])
def test_tiled_deferred_layer_mean_bit_exact(case, rows_per_block):
    """The headline schedule (F.lightgcn_hop_schedule, deferred): y1 parked in the output rows,
    the mean formed on hop 3 from x0, y1 and hop 3's own input rows (EPI_ACC_X) — the
    reference's layer mean, bit for bit."""
    f, g, x0, _, _ = case
    plan = g.tiled_plan(rows_per_block=rows_per_block)
    out = torch.full_like(x0, float("nan"))
    bufs = {"x0": x0, "acc": out, "a": torch.empty_like(x0), "b": torch.empty_like(x0),
            None: None}
    for xn, yn, epi in F.lightgcn_hop_schedule(3, deferred=True):
        F.spmm_tiled_into(g, bufs[xn], bufs[yn], plan, epi=epi, self_rows=x0, acc=out,
                          acc_div=4.0)
    check_layers(f, [], out)


@pytest.mark.parametrize("light", ["throughput", "latency"])
@pytest.mark.parametrize("launch", ["default", "fork", "two"])
@pytest.mark.parametrize("heavy,slice_len", [(256, 0), (256, 2048), (128, 512), (16, 16)])
def test_csr_knobs_bit_exact(case, light, launch, heavy, slice_len):
    """The round-6 CSR hop knobs (gnnrec_spmm_csr_heavy_f32): the row-parallel chain's
    latency form, the light rows as blocks of the heavy launch (the default on this operand
    with the latency form), the heavy rows forked onto the side stream or in a launch after
    the light rows', and the longest heavy rows as feature slices — every combination the
    reference's bits, per hop (spmm_into) and through the K-hop launch."""
    from src.ops import _lib
    f, g, x0, _, _ = case
    flags = (_lib.CSR_LIGHT_LATENCY if light == "latency" else _lib.CSR_LIGHT_THROUGHPUT) | \
        {"default": 0, "fork": _lib.CSR_FORK, "two": _lib.CSR_TWO_LAUNCHES}[launch]
    saved = F.CSR_FLAGS, F.SPMM_SLICE_LEN
    F.CSR_FLAGS, F.SPMM_SLICE_LEN = flags, slice_len
    try:
        if slice_len:
            assert g.heavy_rows_longer(heavy, slice_len) > 0
        hops, x = [], x0
        for _ in range(3):
            y = torch.empty_like(x0)
            F.spmm_into(g, x, y, heavy_threshold=heavy)
            hops.append(y)
            x = y
        check_layers(f, hops)
        out, layers = F.lightgcn_forward(g, x0, 3, return_layers=True, heavy_threshold=heavy)
        check_layers(f, list(layers), out)
        out2, _ = F.lightgcn_forward(g, x0, 3, heavy_threshold=heavy)
        assert torch.equal(out, out2)
    finally:
        F.CSR_FLAGS, F.SPMM_SLICE_LEN = saved


@pytest.mark.parametrize("d", [32, 128, 256])
def test_sliced_heavy_rows_other_widths(case, d):
    """Feature slices at the other sliced instances (d/2 = 16, 64, 128 features per slice),
    with the fork: the same bits as the unsplit row-parallel kernel (heavy=0), which the d=64
    case pins to the reference."""
    from src.ops import _lib
    _, g, _, _, _ = case
    x = torch.randn(g.shape[1], d, device=g.device,
                    generator=torch.Generator(device=g.device).manual_seed(d))
    ref = torch.empty(g.n_rows, d, device=g.device)
    F.spmm_into(g, x, ref, heavy_threshold=0)
    saved = F.CSR_FLAGS, F.SPMM_SLICE_LEN
    try:
        for flags, sl in ((0, 1024), (0, 2048), (_lib.CSR_TWO_LAUNCHES, 2048),
                          (_lib.CSR_FORK, 256), (_lib.CSR_FORK, 0)):
            F.CSR_FLAGS, F.SPMM_SLICE_LEN = flags, sl
            y = torch.full_like(ref, float("nan"))
            F.spmm_into(g, x, y, heavy_threshold=256)
            assert torch.equal(y, ref), (flags, sl)
    finally:
        F.CSR_FLAGS, F.SPMM_SLICE_LEN = saved


def test_sliced_heavy_rows_large_operand(cuda):
    """Above 65 536 rows the d = 64 heavy rows slice into two 32-feature (whole-line) pieces,
    and the row-parallel kernel's form follows the light rows' degree (functional
    light_form_flag: this operand's light rows are short, so the latency form): a 100K-row
    power-law operand with rows of several thousand neighbours, every knob combination — both
    light-row forms forced, the fork — bit-identical to the plain row-parallel chain
    (heavy=0), at d = 64 and 128."""
    from src.ops import _lib
    rng = np.random.default_rng(11)
    nu, ni, n = 60_000, 40_000, 1_500_000
    items = np.minimum((rng.zipf(1.6, n) - 1), ni - 1)
    users = rng.integers(0, nu, n)
    g = CsrGraph.from_interactions(users, items, nu, ni).to(cuda)
    assert g.n_rows > 65_536 and g.max_degree() > 4096
    assert F.light_form_flag(g, 128) & _lib.CSR_LIGHT_LATENCY
    saved = F.CSR_FLAGS, F.SPMM_SLICE_LEN
    try:
        for d in (64, 128):
            x = torch.randn(g.shape[1], d, device=cuda,
                            generator=torch.Generator(device=cuda).manual_seed(d))
            ref = torch.empty(g.n_rows, d, device=cuda)
            F.spmm_into(g, x, ref, heavy_threshold=0)
            for flags, sl, ht in ((0, 1024, 128), (0, 0, 256), (_lib.CSR_LIGHT_LATENCY, 512, 256),
                                  (_lib.CSR_LIGHT_THROUGHPUT, 4096, 256),
                                  (_lib.CSR_FORK, 1024, 128)):
                F.CSR_FLAGS, F.SPMM_SLICE_LEN = flags, sl
                y = torch.full_like(ref, float("nan"))
                F.spmm_into(g, x, y, heavy_threshold=ht)
                assert torch.equal(y, ref), (d, flags, sl, ht)
    finally:
        F.CSR_FLAGS, F.SPMM_SLICE_LEN = saved
