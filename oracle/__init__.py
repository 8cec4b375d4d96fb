"""CPU oracle of the reference propagation path — TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as
the checker. The product package (gnn-recommendations_amd/) never imports this module.

* oracle.c (compiled to _build/liboracle.so with gcc): scalar restatements of the
  reference functions in their arithmetic order (see its header for the citations).
* torch_ref.py: the reference CPU path op for op in plain PyTorch (COO torch.sparse.mm),
  used as the timed CPU baseline ("port") in bench.py.

Pinning: tests/test_oracle.py checks these against tests/golden/*.npz, golden vectors made
by tests/golden/make_golden.py importing the reference itself in the build container.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SRC = HERE / "oracle.c"
SO = HERE / "_build" / "liboracle.so"
CFLAGS = ["-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared", "-fopenmp"]

_lib = None


def build(force: bool = False) -> Path:
    if force or not SO.exists() or SO.stat().st_mtime < SRC.stat().st_mtime:
        SO.parent.mkdir(parents=True, exist_ok=True)
        subprocess.run(["gcc", *CFLAGS, str(SRC), "-o", str(SO), "-lm"], check=True)
    return SO


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = C.CDLL(str(SO))
        _lib.oracle_build_coo_sorted.restype = C.c_int64
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else C.c_void_p(0)


def build_graph(users, items, n_users, n_items, self_loop=False):
    """(row_ptr, col, cnt, deg) of build_bipartite_graph + tocsr (graph_builder.py:49-107)."""
    u = np.ascontiguousarray(users, dtype=np.int64)
    i = np.ascontiguousarray(items, dtype=np.int64)
    N = n_users + n_items
    cap = max(1, 2 * u.size + (N if self_loop else 0))
    rp = np.zeros(N + 1, np.int64)
    col = np.zeros(cap, np.int32)
    cnt = np.zeros(cap, np.float32)
    deg = np.zeros(max(N, 1), np.float32)
    nnz = lib().oracle_build_coo_sorted(_p(u), _p(i), C.c_int64(u.size), C.c_int64(n_users),
                                        C.c_int64(n_items), C.c_int(int(self_loop)), _p(rp),
                                        _p(col), _p(cnt), _p(deg))
    return rp, col[:nnz].copy(), cnt[:nnz].copy(), deg[:N].copy()


def dis_symmetric(deg):
    """np.power(max(deg, 1), -0.5) in float32 (graph_builder.py:111-120)."""
    d = np.maximum(np.asarray(deg, np.float32), np.float32(1.0))
    return np.power(d, np.float32(-0.5)).astype(np.float32)


def normalize_sym(rp, col, cnt, dis):
    val = np.zeros(max(1, col.size), np.float32)
    lib().oracle_normalize_sym(_p(rp), _p(col), _p(_f32(cnt)), C.c_int64(rp.size - 1),
                               _p(_f32(dis)), _p(val))
    return val[:col.size].copy()


def normalized_graph(users, items, n_users, n_items, self_loop=False):
    rp, col, cnt, deg = build_graph(users, items, n_users, n_items, self_loop)
    return rp, col, normalize_sym(rp, col, cnt, dis_symmetric(deg))


def spmm(rp, col, val, x):
    x = _f32(x)
    n = rp.size - 1
    y = np.zeros((n, x.shape[1]), np.float32)
    lib().oracle_spmm(_p(rp), _p(np.ascontiguousarray(col, np.int32)), _p(_f32(val)),
                      C.c_int64(n), _p(x), C.c_int64(x.shape[1]), C.c_int(x.shape[1]), _p(y),
                      C.c_int64(x.shape[1]))
    return y


def lightgcn(rp, col, val, x0, n_layers, return_layers=False):
    x0 = _f32(x0)
    n, d = x0.shape
    out = np.zeros_like(x0)
    scratch = np.zeros((2, n, d), np.float32)
    layers = np.zeros((n_layers, n, d), np.float32) if return_layers else None
    lib().oracle_lightgcn(_p(rp), _p(np.ascontiguousarray(col, np.int32)), _p(_f32(val)),
                          C.c_int64(n), _p(x0), C.c_int(d), C.c_int(n_layers), _p(scratch),
                          _p(layers), _p(out))
    return (out, layers) if return_layers else out


def gas(x, blocks, perm):
    x = _f32(x)
    b = _f32(blocks)
    y = np.zeros_like(x)
    lib().oracle_gas(_p(x), C.c_int64(x.shape[0]), C.c_int(x.shape[1]), C.c_int(b.shape[1]),
                     _p(b), _p(np.ascontiguousarray(perm, np.int32)), _p(y))
    return y


def ngcf_layer(rp, col, val, x, W1, b1, W2, b2, slope=0.2):
    x = _f32(x)
    n, d = x.shape
    nbuf = np.zeros_like(x)
    out = np.zeros_like(x)
    lib().oracle_ngcf_layer(_p(rp), _p(np.ascontiguousarray(col, np.int32)), _p(_f32(val)),
                            C.c_int64(n), _p(x), C.c_int(d), _p(_f32(W1)), _p(_f32(b1)),
                            _p(_f32(W2)), _p(_f32(b2)), C.c_float(slope), _p(nbuf), _p(out))
    return out


def score_topk(u, v, k, seen_ptr=None, seen_col=None):
    u, v = _f32(u), _f32(v)
    nb = u.shape[0]
    idx = np.zeros((nb, k), np.int64)
    sc = np.zeros((nb, k), np.float32)
    sp_ = None if seen_ptr is None else np.ascontiguousarray(seen_ptr, np.int64)
    sc_ = None if seen_col is None else np.ascontiguousarray(seen_col, np.int32)
    lib().oracle_score_topk(_p(u), C.c_int64(nb), _p(v), C.c_int64(v.shape[0]),
                            C.c_int(u.shape[1]), _p(sp_), _p(sc_), C.c_int(k), _p(idx), _p(sc))
    return idx, sc


def gat_head(rp, col, h, ss, sn, slope=0.2):
    """One head of the GAT aggregation; h: [N, o], ss/sn: [N]. float64 accumulation."""
    h = _f32(h)
    if h.shape[1] > 1024:
        raise ValueError("oracle.gat_head: o_dim <= 1024")
    ss, sn = _f32(ss).reshape(-1), _f32(sn).reshape(-1)
    n = rp.size - 1
    out = np.zeros((n, h.shape[1]), np.float32)
    lib().oracle_gat_head(_p(rp), _p(np.ascontiguousarray(col, np.int32)), C.c_int64(n), _p(h),
                          C.c_int64(h.shape[1]), _p(ss), _p(sn), C.c_int64(1),
                          C.c_int(h.shape[1]), C.c_float(slope), _p(out), C.c_int64(h.shape[1]))
    return out
