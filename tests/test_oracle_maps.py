"""Oracle integer maps vs fixtures generated from the reference itself (bit-exact)."""
import numpy as np
import pytest
import torch

from oracle.index_maps import shifted_window_rows, shift_mask, relative_position_index, relative_coords_table

CASES = [((12, 12), 6), ((12, 18), 6), ((84, 84), 6), ((6, 6), 3)]


@pytest.mark.parametrize("hw,ws", CASES)
def test_rows_match_reference(golden, hw, ws):
    g = golden("maps.npz")
    for s in (0, ws // 2):
        ref = g[f"rows_{hw[0]}x{hw[1]}_ws{ws}_s{s}"]
        got = shifted_window_rows(2, hw, (ws, ws), (s, s))
        assert got.dtype == np.int64
        np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("hw,ws", CASES)
def test_mask_matches_reference(golden, hw, ws):
    ref = golden("maps.npz")[f"mask_{hw[0]}x{hw[1]}_ws{ws}_s{ws // 2}"]
    got = shift_mask(hw, (ws, ws), (ws // 2, ws // 2))
    np.testing.assert_array_equal(got, ref)


def test_swin_v2_mask_matches_reference(golden):
    ref = golden("maps.npz")["v2mask_12x12_ws6_s3"]
    np.testing.assert_array_equal(shift_mask((12, 12), (6, 6), (3, 3)), ref)


@pytest.mark.parametrize("ws", [6, 3, 4])
def test_relative_index_matches_reference(golden, ws):
    np.testing.assert_array_equal(relative_position_index((ws, ws)), golden("maps.npz")[f"relidx_ws{ws}"])


@pytest.mark.parametrize("ws", [6, 3, 4])
def test_coords_table_matches_reference(golden, ws):
    ref = golden("maps.npz")[f"coords_ws{ws}"]
    got = relative_coords_table((ws, ws))
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-7)


def test_3d_maps_reduce_to_2d():
    """The dimension-generic maps at D = 1 (window depth 1) equal the 2D maps."""
    r2 = shifted_window_rows(2, (12, 18), (6, 6), (3, 3))
    r3 = shifted_window_rows(2, (1, 12, 18), (1, 6, 6), (0, 3, 3))
    np.testing.assert_array_equal(r2, r3)
    np.testing.assert_array_equal(shift_mask((12, 18), (6, 6), (3, 3)), shift_mask((1, 12, 18), (1, 6, 6), (0, 3, 3)))
    np.testing.assert_array_equal(relative_position_index((6, 6)), relative_position_index((1, 6, 6)))


def test_3d_rows_are_a_permutation():
    rows = shifted_window_rows(2, (12, 12, 12), (6, 6, 6), (3, 3, 3))
    assert rows.shape == (2 * 8, 216)
    np.testing.assert_array_equal(np.sort(rows.reshape(-1)), np.arange(2 * 12 ** 3))


def test_3d_mask_region_count():
    """3D shifted mask: 8 windows per 12^3 volume; the corner window mixes 2^3 regions."""
    m = shift_mask((12, 12, 12), (6, 6, 6), (3, 3, 3))
    assert m.shape == (8, 216, 216)
    assert (m[0] == 0).all()          # interior window: single region
    last = m[-1]                        # corner window: 8 regions of 27 tokens each
    assert ((last == 0).sum(axis=1) == 27).all()


@pytest.mark.parametrize("res,window,shift", [((12, 18), (6, 6), (3, 3)), ((84, 84), (6, 6), (3, 3)),
                                              ((12, 12, 18), (6, 6, 6), (3, 3, 3)), ((1, 12, 12), (1, 6, 6), (0, 2, 2))])
def test_mask_geometry_recovered_from_calculate_mask(res, window, shift):
    """The reference-signature path (forward(x_windows, mask)) maps a calculate_mask back to a
    geometry whose analytic mask is identical."""
    from multimodal_neuroimage_amd.modules._common import geometry_for_mask, shift_mask_buffer
    mask = shift_mask_buffer(res, window, shift)
    got = geometry_for_mask(mask, window)
    assert got is not None
    assert torch.equal(shift_mask_buffer(got[0], window, got[1]), mask)
    assert geometry_for_mask(torch.randn(mask.shape), window) is None


def test_mask_geometry_cache_is_keyed_on_the_live_tensor():
    """a cached geometry must never be returned for a different mask that reuses a freed
    mask's identity, nor for a mask mutated in place; the cache stays bounded; an all-zero mask (an
    unshifted layer) maps to shift 0."""
    from multimodal_neuroimage_amd.modules import _common as Cm
    window = (6, 6)
    a = Cm.shift_mask_buffer((12, 12), window, (3, 3))
    b = Cm.shift_mask_buffer((12, 12), window, (2, 2))
    assert Cm.geometry_for_mask(a, window)[1] == (3, 3)
    # same tensor object rewritten in place: a new version, recomputed
    a.copy_(b)
    assert Cm.geometry_for_mask(a, window)[1] == (2, 2)
    # a stale entry (its tensor freed) is never served to another tensor, even one with the same key
    key = next(reversed(Cm._MASK_GEOMETRY))
    Cm._MASK_GEOMETRY[key] = (lambda: None, ((99, 99), (5, 5)))
    assert Cm.geometry_for_mask(a, window)[1] == (2, 2)
    for _ in range(3 * Cm._MASK_GEOMETRY_MAX):
        Cm.geometry_for_mask(Cm.shift_mask_buffer((12, 12), window, (3, 3)), window)
    assert len(Cm._MASK_GEOMETRY) <= Cm._MASK_GEOMETRY_MAX
    z = torch.zeros(4, 36, 36)
    res, shift = Cm.geometry_for_mask(z, window)
    assert shift == (0, 0) and torch.equal(Cm.shift_mask_buffer(res, window, shift), z)
