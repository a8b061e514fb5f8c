"""Workgroup -> work maps restated in Python and checked on CPU:

* kcommon.h span_pair: the stamp shards of a launch;
* k_gemm.hip gemm_splitk / splitk_factor: every 32-deep k-step of every
  Whisper width covered exactly once by the split-K slices and waves.
"""
import pytest


def test_span_shards_spread_over_eight_pairs():
    SPAN_SHARDS = 8
    offs = {(wg % SPAN_SHARDS) * 16 for wg in range(640)}
    assert offs == {16 * s for s in range(SPAN_SHARDS)}
    assert all(o % 16 == 0 for o in offs)  # 128-B apart (u64 index x 8 bytes)


def splitk_factor(K):
    """k_gemm.hip splitk_factor (MWX_SPLITK_KSMAX unset)."""
    if K % 128:
        return 0
    S = K // 32
    for ks in range(8, 0, -1):
        if S % ks == 0 and (S // ks) % 4 == 0 and (S // ks) // 4 <= 5:
            return ks
    return 0


@pytest.mark.parametrize("K", [384, 512, 768, 1024, 1280, 1536, 2048, 3072, 4096, 5120])
def test_splitk_slices_cover_k_once(K):
    ks = splitk_factor(K)
    assert ks > 0
    kslice, kch = K // ks, K // ks // 128
    assert 1 <= kch <= 5
    steps = []
    for s in range(ks):
        for wid in range(4):  # 4 waves per workgroup, kch k-steps each
            kt0 = (s * kslice >> 5) + wid * kch
            steps.extend(range(kt0, kt0 + kch))
    assert sorted(steps) == list(range(K // 32))
