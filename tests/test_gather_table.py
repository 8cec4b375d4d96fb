"""Placement of the tables the package allocates for its own gathered blocks
(functional.gather_table; the slow 128-B line offset measured in profiles/r04/)."""
import torch

from src.ops import functional as F


def _lines(addr, cols, esz=4):
    return [(addr + o) % 1024 for o in range(0, cols * esz, 128)]


def test_shift_keeps_gathered_lines_off_the_slow_offset():
    # config 3: [N, 4 x 64] fp32 rows (1 KB), blocks x0..x2 gathered
    for base in range(0, 1024, 128):
        s = F.gather_table_shift(base, 256, 192)
        assert s is not None and 0 <= s < 256
        assert F.SLOW_GATHER_LINE not in _lines(base + 4 * s, 192)
    assert F.gather_table_shift(0, 256, 192) == 128        # 512 B: blocks at 512, 768, 0
    # nothing to choose: rows not a multiple of 1 KB apart, unaligned, every offset gathered
    assert F.gather_table_shift(0, 64, 64) is None
    assert F.gather_table_shift(64, 256, 192) is None
    assert F.gather_table_shift(0, 512, 384) is None
    # already clear: no shift
    assert F.gather_table_shift(0, 256, 64) == 0


def test_gather_table_is_a_contiguous_view_of_the_requested_shape():
    for n, w, g in ((1000, 256, 192), (10, 64, 64), (0, 256, 192), (7, 512, 256)):
        t = F.gather_table(n, w, g)
        assert t.shape == (n, w) and t.is_contiguous() and t.dtype == torch.float32
        if n:
            t.fill_(1.0)
            assert float(t.sum()) == n * w
            shift = F.gather_table_shift(t.untyped_storage().data_ptr(), w, g)
            if shift is not None:
                assert t.storage_offset() == shift


def test_hop_table_layout_keeps_every_row_line_off_the_slow_offset():
    for d, (ld, start) in F.HOP_TABLE_LAYOUT.items():
        t = F.hop_table(64, d, zero=True)
        assert t.shape == (64, d) and t.stride() == (ld, 1)
        assert float(t.abs().sum()) == 0.0
        base = t.data_ptr()
        if base % 128 == 0:      # placement is by the actual address
            assert (base - start) % 1024 == 0
            for r in range(64):
                assert F.SLOW_GATHER_LINE not in _lines(base + 4 * ld * r, d)
    t = F.hop_table(5, 48)       # no layout for this width: a compact tensor
    assert t.is_contiguous() and t.shape == (5, 48)
