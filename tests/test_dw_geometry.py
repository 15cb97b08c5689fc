"""Host-side depthwise tile geometry (no GPU needed: the partial counts are computed by the
launchers' geometry code in the extension).  The BN-statistics and weight-gradient workspaces
are sized from these counts, so they must follow every geometry switch: tall strips across
image boundaries on <= 14-row stride-1 maps (csrc/kernels/dwconv.hip dw_geom), the round-aware
small-map dgrad choice; the weight gradient keeps per-image strips."""
import pytest

import pgdist  # noqa: F401
from pgdist.ops import kernels as K


@pytest.fixture
def geom():
    old = (K.dw_tall_rows(), K.dw_small_dgrad(), K.dw_geom_mode())
    yield
    K.dw_set_tall_rows(old[0])
    K.dw_set_small_dgrad(old[1])
    K.dw_set_geom_mode(old[2])


def test_tall_forward_strips_span_images(geom):
    K.dw_set_tall_rows(0)
    assert K.dw_num_partials("fwd", 128, 7, 7, 960, 1) == 128        # one strip per 7x7 image
    K.dw_set_tall_rows(14)
    assert K.dw_num_partials("fwd", 128, 7, 7, 960, 1) == 64         # two images per strip
    assert K.dw_num_partials("fwd", 5, 7, 7, 960, 1) == 3            # 35 rows: a partial last strip
    K.dw_set_tall_rows(10)
    assert K.dw_num_partials("fwd", 5, 7, 7, 960, 1) == 4            # strips starting mid-image


def test_tall_leaves_other_layers_alone(geom):
    K.dw_set_tall_rows(0)
    s2 = [K.dw_num_partials(k, 128, 14, 14, 576, 2) for k in ("fwd", "dgrad")]
    for rows in (14, 28):
        K.dw_set_tall_rows(rows)
        # stride 2 and a single image keep the per-image tiling
        assert [K.dw_num_partials(k, 128, 14, 14, 576, 2) for k in ("fwd", "dgrad")] == s2
        assert K.dw_num_partials("fwd", 1, 7, 7, 960, 1) == 1
    # maps > 14 rows too
    K.dw_set_tall_rows(0)
    ref = [K.dw_num_partials(k, 128, 28, 28, 192, s) for k in ("fwd", "dgrad", "wgrad") for s in (1, 2)]
    K.dw_set_tall_rows(14)
    assert [K.dw_num_partials(k, 128, 28, 28, 192, s) for k in ("fwd", "dgrad", "wgrad") for s in (1, 2)] == ref


def test_round_aware_small_dgrad(geom):
    K.dw_set_tall_rows(14)
    K.dw_set_small_dgrad(0)
    assert K.dw_num_partials("dgrad", 128, 14, 14, 576, 1) == 128     # 72-channel slabs, 1024 workgroups
    K.dw_set_small_dgrad(1)
    assert K.dw_num_partials("dgrad", 128, 14, 14, 576, 1) == 86      # 21-row strips: ceil(1792 / 21)
    assert K.dw_num_partials("dgrad", 128, 14, 14, 384, 1) == 128     # 64-channel slabs of all 14 columns
    # the fused dgrad + wgrad workspace follows the dgrad partial count
    P = K.dw_num_partials("dgrad", 128, 14, 14, 576, 1)
    assert K.dw_dgrad_wgrad_workspace(128, 14, 14, 576, 1) >= P * 9 * 576


def test_weight_gradient_keeps_per_image_strips(geom):
    for rows in (0, 14):
        K.dw_set_tall_rows(rows)
        assert K.dw_num_partials("wgrad", 128, 7, 7, 960, 1) == 128
