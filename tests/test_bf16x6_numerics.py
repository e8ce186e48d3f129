"""CPU restatement of the bf16x6 split (csrc/dense.hip split3, used by gcg_gemm_nt_f32_bf16x6 and
the fused output layer): an f32 x is split into three bf16 planes, each the round-to-nearest-even
bf16 of what the planes before it left; a product a . b keeps the six plane products of order
<= 2^-16. These tests pin the numerical claims the kernels' docs make, on numpy float64 sums of
the same planes (the MFMA forms each plane product exactly in f32). Range: magnitudes 1e-30 to
1e30; below ~2^-109 the third plane is subnormal in f32 (a flushing MFMA would lose it: the
product's relative error can then reach 2^-16, still far below the float64 bars of the GPU tests
for activations and weights of a trained layer)."""
import numpy as np
import pytest


def bf16_rne(x: np.ndarray) -> np.ndarray:
    """float32 -> nearest-even bfloat16, returned as float32 (v_cvt_pk_bf16_f32 on finite x)."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    rounded = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return rounded.astype(np.uint32).view(np.float32)


def split3(x: np.ndarray):
    x = x.astype(np.float32)
    h0 = bf16_rne(x)
    r1 = (x - h0).astype(np.float32)  # exact in f32
    h1 = bf16_rne(r1)
    r2 = (r1 - h1).astype(np.float32)
    h2 = bf16_rne(r2)
    return h0, h1, h2


def _values(n, seed):
    rng = np.random.default_rng(seed)
    return (rng.choice([-1.0, 1.0], n) * 10.0 ** rng.uniform(-30, 30, n)).astype(np.float32)


def test_bf16_rne_matches_round_half_even():
    x = np.array([1.0, 1.00390625, 1.005859375, 1.0078125, -2.00390625, 3.0e38], np.float32)
    got = bf16_rne(x)
    # 1 + 2^-8 is a tie (rounds to even: 1.0), 1 + 1.5 * 2^-8 rounds up to 1 + 2^-7
    assert got[0] == 1.0 and got[1] == 1.0 and got[2] == np.float32(1.0078125)
    assert got[3] == np.float32(1.0078125) and got[4] == np.float32(-2.0)
    assert np.all(got.view(np.uint32) & 0xFFFF == 0)


def test_three_planes_reconstruct_f32():
    x = _values(200_000, 1)
    h0, h1, h2 = split3(x)
    for h in (h0, h1, h2):
        assert np.all(h.view(np.uint32) & 0xFFFF == 0)  # each plane is a bf16 value
    rec = h0.astype(np.float64) + h1 + h2
    # 3 x 8 significant bits hold the 24-bit f32 significand: exact (gcg_spmm.h)
    assert np.array_equal(rec, x.astype(np.float64))
    # plane magnitudes (gcg_spmm.h): |x1| <= 2^-8 |x| (a half-ulp of an 8-bit significand at the
    # bottom of a binade), |x2| <= 2^-17 |x|
    assert (np.abs(h1) <= 2.0 ** -8 * np.abs(x)).all()
    assert (np.abs(h2) <= 2.0 ** -17 * np.abs(x)).all()


@pytest.mark.parametrize("seed", [2, 3])
def test_six_products_within_f32_rounding(seed):
    """a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0 against the exact product: the dropped terms
    a1b2 + a2b1 + a2b2 stay below (2^-24 + 2^-34) |ab| -- the bound gcg_spmm.h states, one f32
    rounding of the product (measured max ~2^-24.2)."""
    a, b = _values(200_000, seed), _values(200_000, seed + 10)
    a0, a1, a2 = (h.astype(np.float64) for h in split3(a))
    b0, b1, b2 = (h.astype(np.float64) for h in split3(b))
    six = a0 * b0 + a0 * b1 + a1 * b0 + a0 * b2 + a1 * b1 + a2 * b0
    exact = a.astype(np.float64) * b.astype(np.float64)
    rel = np.abs(six - exact) / np.abs(exact)
    assert rel.max() <= 2.0 ** -24 + 2.0 ** -34


def test_nan_reaches_every_plane():
    h0, h1, h2 = split3(np.array([np.nan, 1.5], np.float32))
    assert np.isnan(h0[0]) and np.isnan(h1[0]) and np.isnan(h2[0])
    assert h0[1] == 1.5 and h1[1] == 0.0 and h2[1] == 0.0
