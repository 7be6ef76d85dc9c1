"""The oracle's deliberate RNG-side deviations pinned at image level.

The restatement (and the kernel, bit for bit) draws RandUnitVec3 / RandInUnitDisk by inverse-CDF
maps, ConstantMedium's log by the float polynomial LogU, the marble sin in double and Schlick's
x^5 as a product. The oracle control CTL_REF_MATH puts back the reference's own forms
(Math.hpp:26-43 rejection loops on the same Philox stream, ConstantMedium.cpp:42 std::log,
Texture.cpp:16 std::sin(float), Material.cpp:24 glm::pow = std::pow(double, int)). Converged images of
the two must differ by no more than two seeds of the default oracle do (tools/refmath_pin.py has the
statistics; DESIGN.md §2 records them at 128^2 @ 1024 spp). Bounds, fixed before measuring:
|z_mean| < 4 (a 4-sigma difference of the image means) and the robust per-pixel noise ratio r_mad
within 10 % of 1.
"""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
from refmath_pin import compare  # noqa: E402


@pytest.mark.parametrize("name,spp", [("cornell_box_original", 1024), ("cornell_box_volume", 1024),
                                      ("book2_final_scene_10000_samples", 512)])
def test_reference_math_matches_default_oracle(name, spp):
    r = compare(name, 64, spp)
    assert abs(r["z_mean"]) < 4.0, r
    assert 0.9 < r["r_mad"] < 1.1, r


def test_reference_math_control_changes_the_stream():
    """The control is wired: rejection sampling consumes the stream differently (a cheap check that
    the comparison above is not of two identical images)."""
    import numpy as np
    from refmath_pin import render
    from oracle.oracle import CTL_REF_MATH
    a, _ = render("cornell_box_original", 16, 4, 5, 0)
    b, _ = render("cornell_box_original", 16, 4, 5, CTL_REF_MATH)
    assert not np.array_equal(a, b)
