"""The real-shape reference fixtures on the CPU (BASELINE configs 3 and 5 at config 2's and a
power-law graph's shapes): the drop-in classes, rebuilt from the reference's seeds, give the
reference's own outputs through their CPU path (the reference's torch ops on a torch COO
operand). This pins the fixtures and the model construction the GPU tests
(tests/test_real_shapes_gpu.py) rely on."""
import numpy as np
import torch

from real_shapes import gat_heavy, ml1m_graph, ngcf_ml1m, ob_ml1m


def test_ngcf_ml1m_cpu_matches_reference():
    adj = ml1m_graph().to_torch_sparse_coo()
    for gas in (False, True):
        m, f = ngcf_ml1m(gas)
        with torch.no_grad():
            u, i = m(adj)
        out = torch.cat([u, i]).numpy()[f["rows"]]
        np.testing.assert_allclose(out, f["out_rows"], rtol=1e-6, atol=1e-6, err_msg=f"gas={gas}")


def test_ob_ml1m_cpu_matches_reference():
    adj = ml1m_graph().to_torch_sparse_coo()
    m, f = ob_ml1m()
    with torch.no_grad():
        u, i = m(adj_matrix=adj)
        layers = m.get_layer_embeddings(adj_matrix=adj)
    np.testing.assert_allclose(torch.cat([u, i]).numpy()[f["rows"]], f["out_rows"], rtol=1e-6,
                               atol=1e-6)
    for k in range(4):
        np.testing.assert_allclose(layers[k].numpy()[f["rows"]], f["layers_rows"][k], rtol=1e-6,
                                   atol=1e-6)


def test_gat_heavy_fixture_shape():
    """The power-law fixture really exercises the degree-bucketed path (rows > 2048), and the
    CPU path (the reference's dense masked softmax) reproduces it."""
    from src.ops import functional as F
    m, f, g = gat_heavy()
    deg = np.diff(g.row_ptr.numpy())
    assert int((deg > F.GAT_LARGE_KNOBS[0]).sum()) >= 2 and deg.min() >= 1
    with torch.no_grad():
        u, i = m(g.to_torch_sparse_coo())
    np.testing.assert_allclose(u.numpy(), f["user_out"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(i.numpy(), f["item_out"], rtol=1e-5, atol=1e-6)
