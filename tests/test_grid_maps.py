"""Workgroup -> work maps of the launch layouts, restated in Python and checked
on CPU (the kernels themselves are checked bit-identical against the
separate launches by the -m gpu tests, tests/test_gpu_chain.py):

* k_chain.hip chain_kernel: the three block roles of a chained decode seam
  (producer split-K GEMM tiles, one LayerNorm block per row, consumer GEMM
  tiles) cover their work exactly once; every hand-off counter receives
  exactly the arrivals its waiters wait for; and every block waits only for
  blocks of lower id (so in-order dispatch can never leave a waiter without
  its producers);
* kcommon.h span_pair: the stamp shards of a launch.
"""
import itertools

import pytest


def splitk_factor(K):
    """k_gemm.hip splitk_factor (MWX_SPLITK_KSMAX unset)."""
    if K % 128:
        return 0
    S = K // 32
    for ks in range(8, 0, -1):
        if S % ks == 0 and (S // ks) % 4 == 0 and (S // ks) // 4 <= 5:
            return ks
    return 0


def chain_blocks(M, d, prod_K, c_N, skinny):
    """chain_kernel's role of every block id, as chain_launch sizes the grid:
    ('P', bx, ks, bz) | ('L', row) | ('CS', bx, ks, bz) | ('CK', bx, by)."""
    nrb = (M + 15) // 16
    nx = (d + 15) // 16
    p_ks = splitk_factor(prod_K) if prod_K else 0
    n1 = nx * p_ks * nrb if prod_K else 0
    nxc = (c_N + 15) // 16
    c_ks = splitk_factor(d)
    nc = nxc * nrb if skinny else nxc * c_ks * nrb
    roles = []
    for b in range(n1 + M + nc):
        if b < n1:
            roles.append(("P", b % nx, (b // nx) % p_ks, b // (nx * p_ks)))
            continue
        b2 = b - n1
        if b2 < M:
            roles.append(("L", b2))
            continue
        b3 = b2 - M
        if skinny:
            roles.append(("CK", b3 % nxc, b3 // nxc))
        else:
            roles.append(("CS", b3 % nxc, (b3 // nxc) % c_ks, b3 // (nxc * c_ks)))
    return roles, p_ks, c_ks, nx, nxc, nrb


SHAPES = [  # (M rows, d, producer K (0: none), consumer N, skinny consumer)
    (32, 1280, 1280, 1280, False),   # out-proj -> LN2 -> cross-Q (large-v3, 32 rows)
    (32, 1280, 1280, 5120, True),    # cross-out -> LN3 -> FFN1
    (32, 1280, 5120, 3840, False),   # FFN2 -> LN1 -> QKV
    (32, 1280, 0, 3840, False),      # (layer 0) LN1 -> QKV
    (1, 512, 2048, 1536, False),     # base, one request (C2)
    (1, 512, 512, 2048, True),
    (5, 384, 1536, 1152, False),     # tiny, a few rows
    (64, 1024, 4096, 3072, False),   # medium, 64 rows
    (17, 128, 512, 512, True),       # micro, a partial row block
]


@pytest.mark.parametrize("M,d,pK,cN,skinny", SHAPES)
def test_chain_roles_cover_work_once(M, d, pK, cN, skinny):
    roles, p_ks, c_ks, nx, nxc, nrb = chain_blocks(M, d, pK, cN, skinny)
    prods = [r for r in roles if r[0] == "P"]
    lns = [r for r in roles if r[0] == "L"]
    cons = [r for r in roles if r[0] in ("CS", "CK")]
    if pK:
        assert sorted(prods) == sorted(("P", x, k, z) for x in range(nx) for k in range(p_ks)
                                       for z in range(nrb))
    assert sorted(r[1] for r in lns) == list(range(M))
    if skinny:
        assert sorted(cons) == sorted(("CK", x, y) for x in range(nxc) for y in range(nrb))
    else:
        assert sorted(cons) == sorted(("CS", x, k, z) for x in range(nxc) for k in range(c_ks)
                                      for z in range(nrb))
    # every K range of the split-K GEMMs is covered exactly once per column strip
    if pK:
        assert (pK // p_ks) * p_ks == pK and (pK // p_ks) % 128 == 0
    if not skinny:
        assert (d // c_ks) * c_ks == d and (d // c_ks) % 128 == 0


@pytest.mark.parametrize("M,d,pK,cN,skinny", SHAPES)
def test_chain_counters_and_wait_order(M, d, pK, cN, skinny):
    roles, p_ks, c_ks, nx, nxc, nrb = chain_blocks(M, d, pK, cN, skinny)
    arrivals_p = [0] * nrb   # producer arrivals per row block
    arrivals_l = [0] * nrb   # LayerNorm arrivals per row block
    last_p = [-1] * nrb      # highest block id that arrives on each counter
    last_l = [-1] * nrb
    for b, r in enumerate(roles):
        if r[0] == "P":
            arrivals_p[r[3]] += 1
            last_p[r[3]] = max(last_p[r[3]], b)
        elif r[0] == "L":
            arrivals_l[r[1] // 16] += 1
            last_l[r[1] // 16] = max(last_l[r[1] // 16], b)
    for b, r in enumerate(roles):
        if r[0] == "L" and pK:
            rb = r[1] // 16
            assert arrivals_p[rb] == nx * p_ks      # the LayerNorm's wait target
            assert last_p[rb] < b                   # producers precede the waiter
        elif r[0] in ("CS", "CK"):
            rb = r[3] if r[0] == "CS" else r[2]
            assert arrivals_l[rb] == min(16, M - 16 * rb)  # the consumer's target
            assert last_l[rb] < b


def test_span_shards_spread_over_eight_pairs():
    SPAN_SHARDS = 8
    offs = {(wg % SPAN_SHARDS) * 16 for wg in range(640)}
    assert offs == {16 * s for s in range(SPAN_SHARDS)}
    assert all(o % 16 == 0 for o in offs)  # 128-B apart (u64 index x 8 bytes)


@pytest.mark.parametrize("d", [128, 256, 384, 512, 768, 1024, 1280])
def test_chain_supports_every_whisper_width(d):
    """chain_launch's shape rules hold for every Whisper width: d % 128 == 0,
    split-K k-steps per wave within 1..5, the skinny FFN1 4-wave split within
    the kernel's 10 k-steps."""
    assert d % 128 == 0 and d <= 2048
    for K in (d, 4 * d):
        ks = splitk_factor(K)
        assert ks > 0 and 1 <= K // ks // 128 <= 5
    assert (d // 32) % 4 == 0 and d // 32 // 4 <= 10
    for M, w in itertools.product([1, 16, 32, 64], [d]):
        assert (M + 15) // 16 <= 4
