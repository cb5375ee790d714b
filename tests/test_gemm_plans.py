"""CPU checks of the GEMM launch planning (no GPU): the 2 GiB DMA-range guards of gemm8 / gemm8w
 evaluated on meta tensors of the production shapes."""

import torch

from cs336_systems.ops import gemm


def _meta(*shape):
    return torch.empty(*shape, device="meta", dtype=torch.bfloat16)


def test_g8w_split_fits_vocab_50304():
    # a 50304-vocabulary head at 49152 tokens: dY is 4.9 GB, a single split cannot be addressed
    dy, x = _meta(49152, 50304), _meta(49152, 1600)
    assert not gemm.g8w_split_fits(49152, 1, dy, x)
    assert not gemm.g8w_split_fits(49152, 2, dy, x)
    assert gemm.g8w_split_fits(49152, 4, dy, x)  # 12288 rows x 100 KB < 2 GiB
    trans, sk = gemm.dw_launch_plan(dy, x)
    assert sk == 1 or gemm.g8w_split_fits(49152, sk, dy, x)


def test_g8w_split_fits_xl_shapes():
    for n_out, k_in in ((12800, 1600), (1600, 6400), (4800, 1600), (1600, 1600), (10000, 1600)):
        dy, x = _meta(49152, n_out), _meta(49152, k_in)
        _, sk = gemm.dw_launch_plan(dy, x)
        assert sk == gemm._dw_plan(49152, n_out, k_in)[1]  # the measured plans are unchanged
    # 2.7b W1|W3 past ~52k tokens: one split of 20480-wide rows no longer fits
    assert not gemm.g8w_split_fits(65536, 1, _meta(65536, 20480), _meta(65536, 2560))


def test_gemm8_extents():
    assert gemm.gemm8_extents_ok(_meta(49152, 10000), _meta(1600, 10000))
    assert gemm.gemm8_extents_ok(_meta(49152, 1600), _meta(10000, 1600))
    assert not gemm.gemm8_extents_ok(_meta(4096, 1600), _meta(700000, 1600))


def test_dense_key_matches_table_entry():
    """A problem whose operands sit in wider buffers (ZeRO-1 flat buffers give a group's Wᵀ a row
    stride of 665360 on the 2.7b) maps to the committed dense-layout entry."""
    key = ("nt", (12288, 20480), (20480, 1), (2560, 20480), (665360, 1), None)
    dense = gemm._dense_key(key)
    assert dense == ("nt", (12288, 20480), (20480, 1), (2560, 20480), (20480, 1), None)
    table = gemm.selection_table() if False else __import__("json").load(open(gemm.TABLE_FILE))["entries"]
    assert str(dense) in table
    for k in (("nt", (12288, 2560), (2560, 1), (2560, 2560), (10240, 1), None),
              ("nt", (12288, 7680), (7680, 1), (2560, 7680), (10240, 1), None)):
        assert str(gemm._dense_key(k)) in table
