"""Workgroup -> work maps of the round-3 launch layouts, restated in Python
and checked for coverage on CPU (the kernels themselves are checked
bit-identical against the old layouts by the -m gpu tests):

* k_gemm.hip decode_tile_of: the 1-D grid of the decode GEMMs with the row
  blocks of one weight tile at consecutive ids of one residue mod 8 -- every
  (tile, row block) exactly once, all row blocks of a tile on one residue
  (XCD) and inside one window of 8 x zrb ids;
* k_attn.hip dec_attn_kernel PF: the helper workgroups' K / V chunk ranges
  cover both matrices exactly once;
* kcommon.h span_pair: the stamp shards of a launch.
"""
import itertools

import pytest


def decode_tile_of(L, zrb, ntiles):
    W = 8 * zrb
    w, j = divmod(L, W)
    t = w * 8 + (j & 7)
    return t, j >> 3, t < ntiles


def grid_size(ntiles, zrb):
    return (ntiles + 7) // 8 * 8 * zrb


@pytest.mark.parametrize("ntiles,zrb", list(itertools.product([1, 5, 8, 13, 80, 320, 3241],
                                                               [2, 3, 5, 8])))
def test_decode_tile_map_is_a_bijection_per_xcd(ntiles, zrb):
    seen = {}
    for L in range(grid_size(ntiles, zrb)):
        t, z, ok = decode_tile_of(L, zrb, ntiles)
        if not ok:
            continue
        assert 0 <= z < zrb
        assert (t, z) not in seen
        seen[(t, z)] = L
    assert len(seen) == ntiles * zrb
    for t in range(ntiles):
        ids = [seen[(t, z)] for z in range(zrb)]
        assert len({i % 8 for i in ids}) == 1          # one XCD
        assert max(ids) - min(ids) < 8 * zrb           # one dispatch window


def test_splitk_tile_index_roundtrip():
    # gemm_splitk: tile t = ks * nx + bx over nx column tiles and nks slices
    nx, nks = 80, 5
    pairs = {(t % nx, t // nx) for t in range(nx * nks)}
    assert pairs == {(x, k) for x in range(nx) for k in range(nks)}


@pytest.mark.parametrize("fixed_len,PF", [(1500, 7), (1500, 3), (448, 7), (1, 7)])
def test_prefetch_helpers_cover_k_and_v_once(fixed_len, PF):
    chunks = fixed_len * 8
    per = (2 * chunks + PF - 1) // PF
    got = []
    for p in range(PF):
        c0 = min(p * per, 2 * chunks)
        c1 = min(c0 + per, 2 * chunks)
        got.extend(range(c0, c1))
    assert got == list(range(2 * chunks))


def test_span_shards_spread_over_eight_pairs():
    SPAN_SHARDS = 8
    offs = {(wg % SPAN_SHARDS) * 16 for wg in range(640)}
    assert offs == {16 * s for s in range(SPAN_SHARDS)}
    assert all(o % 16 == 0 for o in offs)  # 128-B apart (u64 index x 8 bytes)
