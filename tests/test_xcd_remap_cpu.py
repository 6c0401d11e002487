"""Block-to-work remaps of the kernels (cgnn_common.h, evaluated on the host through
``_hip.xcd_remap_table``): every form must be a bijection of the grid, the contiguous
form must give each XCD one contiguous range, and the chunk-interleaved form (the GAT
edge kernels) must give XCD x the chunks x, x + 8, ...  The dispatcher deals blocks to
the 8 XCDs round-robin, so block b runs on XCD b % 8."""
import pytest

from cgnn_amd import native


GRIDS = [1, 7, 8, 9, 100, 511, 512, 513, 4096, 4097, 10000, 70001]


@pytest.mark.parametrize("chunk", [0, 64, 512])
@pytest.mark.parametrize("nwg", GRIDS)
def test_remap_is_a_bijection(nwg, chunk):
    t = native.hip().xcd_remap_table(nwg, chunk)
    assert sorted(t) == list(range(nwg))


@pytest.mark.parametrize("nwg", [8, 100, 4097, 70001])
def test_contiguous_remap_gives_each_xcd_one_range(nwg):
    t = native.hip().xcd_remap_table(nwg, 0)
    for x in range(8):
        ids = [t[b] for b in range(x, nwg, 8)]
        assert ids == list(range(ids[0], ids[0] + len(ids))) if ids else True


@pytest.mark.parametrize("chunk", [64, 512])
def test_chunked_remap_interleaves_chunks_over_xcds(chunk):
    nwg = 8 * chunk * 5 + 123                  # five full rounds and a ragged tail
    t = native.hip().xcd_remap_table(nwg, chunk)
    full = nwg // (8 * chunk) * (8 * chunk)
    for b in range(full):
        c = t[b] // chunk                       # the chunk the block works in
        assert c % 8 == b % 8                  # chunk x, x + 8, ... on XCD x
    for b in range(full, nwg):                  # the tail keeps its ids
        assert t[b] == b
    # within a chunk, consecutive blocks of one XCD take consecutive work
    x = 3
    ids = [t[b] for b in range(x, full, 8)]
    for k in range(0, len(ids), chunk):
        seg = ids[k:k + chunk]
        assert seg == list(range(seg[0], seg[0] + chunk))


def test_unknown_chunk_is_refused():
    with pytest.raises(RuntimeError):
        native.hip().xcd_remap_table(64, 32)
