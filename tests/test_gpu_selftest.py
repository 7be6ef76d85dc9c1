"""The kernel's exact arithmetic shortcuts against their reference form on the GPU (rt2_selftest).

* div_by_inv: the unit-normal axis-aligned quad test divides by the ray's correctly rounded
  reciprocal with one fma correction; it must equal IEEE a / b bit for bit wherever the quad test
  can accept the quotient (|b| > 1e-8, a / b >= tmin).
* aabb_hit_fin: the NaN-free slab test must decide exactly like the reference's swap +
  glm::max/min chain with early exits (AABB.hpp:34-47) for every ray with a finite inverse.
* rcp_nr / sqrt_nr: 1/x and sqrt(x) without the range-scaling steps equal the IEEE results over
  the ranges where the kernel uses them (normalize, ray reciprocals).
* div_by_inv over any quotient with numerators down to 2^-100 (a medium box boundary uses every t;
  the kernel guards smaller numerators back to IEEE division).
* acc_slab: the accelerated-list tree's padded slab test (one fma per bound, +-2^100 for an infinite
  1/d) never culls a box that the exact padded slab test accepts, for rays with direction components
  of +-0 and origins inside the padding band (the fma form with 1/d = inf culled those).
* rcp_nr exhaustively: every float bit pattern in its range (3.7e9 values, both signs) gives IEEE 1/x
  with the hardware reciprocal and two Newton steps.
* div_by_inv's single correction against IEEE a / b over significand pairs: the first 2^36 of the
  2^46 (numerators in [1, 1 + 2^-10)), and every one of the 2^23 numerator significands against 2^17
  divisor significands each (b = 1, b = 2 - 2^-23 and a scrambled stride). All 2^46
  were checked once (profiles/r04_log.md).
* sphere roots by the reciprocal (sphere_t_rec's fast path) against IEEE division on rays from on or
  near a sphere's surface, where a numerator hh -+ sqrt(disc) cancels (down to the subnormal range and
  exact zeros), with every interval kind the kernel uses (the medium's boundary queries accept any
  root); `checked` counts the admitted inputs with a cancelled numerator (ADVICE
  r04).
* sqrt_nr (the square root without range scaling) at the samplers' inputs, 1 - z^2 of the unit-vector
  map and the disk radius u, for every one of the 2^24 uniforms.
"""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("which,n", [(0, 1 << 28), (1, 1 << 26), (2, 1 << 28), (3, 1 << 28), (4, 1 << 26),
                                     (5, 1 << 32), (6, 1 << 36), (7, 1 << 40), (8, 1 << 28),
                                     (9, 1 << 24)],
                         ids=["div_by_inv", "aabb_fin", "rcp_sqrt_nr", "div_by_inv_any_t", "acc_slab_conservative",
                              "rcp_nr_every_float", "div_by_inv_significand_pairs", "div_by_inv_every_numerator",
                              "sphere_roots_cancelled", "sqrt_nr_sampler_inputs"])
def test_selftest(have_gpu, which, n):
    from raytrace2_amd._native import selftest
    bad, checked = selftest(which, n, seed=20241015)
    assert checked > (n // 64 if which == 8 else n // 4)
    assert bad == 0, f"{bad} of {checked} differ"
