"""GPU tests of the HBM-staged levels (wst_staged.h): geometries whose padded planes exceed the
LDS-resident kernels (n > 136) -- BASELINE config c5 (256x256 bands, J=6, L=12 -> 384^2 / 192^2
staged, then 96^2 .. 12^2 in LDS) and a one-staged-level case (128^2, J=5 -> 192^2).

Parity bar as everywhere (parity.TOL, per coefficient k, against the float64 oracle's goldens);
batch / chunking / pooling / order-1 properties are checked against the golden planes placed at
several batch positions, so the c5 oracle (~23 s per plane) is never run at test time.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import kymatio_ref as kr
from parity import TOL, assert_parity

import wst_amd  # noqa: F401
from wst_amd import _lib
from wst_amd.numpy import Scattering2D as NpS
from wst_amd.torch import Scattering2D as ThS

pytestmark = pytest.mark.gpu
PHI0 = np.pi / 3.1415


def golden(name):
    d = load_golden(name)
    return d, d["x_u8"].astype(np.float32) / 255


def forward(plan, x, ws_planes=None, pooled=False):
    B = x.shape[0]
    shape = (B, 2 * plan.K) if pooled else (B, plan.K, plan.Mo, plan.No)
    out = torch.empty(shape, device="cuda")
    n = min(B, ws_planes or plan.preferred_batch())
    ws = torch.empty(plan.workspace_bytes(n), dtype=torch.uint8, device="cuda")
    plan.forward(x.data_ptr(), B, out.data_ptr(), pooled, ws.data_ptr(), ws.numel(),
                 torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("name,M,J,L", [("staged192_gray128_J5_L8", 128, 5, 8),
                                         ("c5_ms256_J6_L12", 256, 6, 12)])
def test_staged_batch_positions_chunking_and_parity(name, M, J, L):
    d, x = golden(name)
    ref = d["S"][0]
    rng = np.random.default_rng(3)
    B = 5
    xs = rng.integers(0, 256, (B, M, M), dtype=np.uint8).astype(np.float32) / 255
    pos = [0, 3, 4]
    for i in pos:
        xs[i] = x[0]
    plan = _lib.Plan(M, M, J, L)
    assert plan.preferred_batch() < 2048          # staged plans bound their chunk
    xt = torch.from_numpy(xs).cuda()
    full = forward(plan, xt)
    small = forward(plan, xt, ws_planes=2)        # 3 chunks: 2 + 2 + 1 planes
    assert torch.equal(full, small), "chunked staged run differs"
    for i in pos:
        assert_parity(full[i].cpu().numpy()[None], ref[None], TOL, f"{name} @ {i}")
    assert torch.isfinite(full).all()


def test_staged_pooled_equals_pooling_of_full_output():
    d, x = golden("staged192_gray128_J5_L8")
    xt = torch.from_numpy(np.concatenate([x, x[:, ::-1].copy(), 0.5 * x], 0)).cuda()
    plan = _lib.Plan(128, 128, 5, 8)
    S = forward(plan, xt).double()
    P = forward(plan, xt, pooled=True).double()
    K = plan.K
    scale = S.abs().amax(dim=(0, 2, 3))
    assert torch.all((P[:, :K] - S.mean(dim=(-2, -1))).abs() <= 1e-6 * scale)
    assert torch.all((P[:, K:] - S.std(dim=(-2, -1), unbiased=False)).abs() <= 1e-6 * scale)


def test_staged_order1_against_oracle():
    x = np.random.default_rng(4).integers(0, 256, (2, 128, 128), dtype=np.uint8).astype(np.float32) / 255
    ref = kr.Scattering2D(J=5, shape=(128, 128), L=4, max_order=1)(x)
    got = NpS(J=5, shape=(128, 128), L=4, max_order=1)(x)
    assert got.shape == ref.shape == (2, 1 + 5 * 4, 4, 4)
    assert_parity(got, ref, TOL, "staged order 1")


def test_c5_full_size_properties():
    """BASELINE config 5 at its stated size (64 patches x 4 bands = 256 planes of 256^2, J=6,
    L=12): size-independent properties over the whole batch (S0 affine; S1/S2 shift-invariant
    and positively homogeneous) + golden parity of the planes carrying the golden input."""
    d, x = golden("c5_ms256_J6_L12")
    rng = np.random.default_rng(12)
    xb = rng.integers(0, 256, (64, 4, 256, 256), dtype=np.uint8).astype(np.float32) / 255
    xb[7, 2] = x[0]
    xb[63, 3] = x[0]
    s = ThS(J=6, shape=(256, 256), L=12)
    xt = torch.from_numpy(xb).cuda()
    S = s(xt)
    assert tuple(S.shape) == (64, 4, 2233, 4, 4)
    assert torch.isfinite(S).all()
    for i, c in [(7, 2), (63, 3)]:
        assert_parity(S[i, c].cpu().numpy()[None], d["S"], TOL, f"c5 golden @ ({i},{c})")
    a, b = 0.5, 0.25
    S2 = s(a * xt + b)
    d0 = (S2[:, :, 0] - (a * S[:, :, 0] + PHI0 * b)).abs().max().item()
    assert d0 <= TOL * S2[:, :, 0].abs().max().item()
    Sd, S2d = S.double(), S2.double()
    scale = (a * Sd[:, :, 1:]).abs().amax(dim=(0, 1, 3, 4))
    err = ((S2d[:, :, 1:] - a * Sd[:, :, 1:]).abs().amax(dim=(0, 1, 3, 4)) / scale).max().item()
    assert err <= 2 * TOL, err


@pytest.mark.parametrize("name,M,N,J,L", [("rectstaged_256x128_J4_L8", 256, 128, 4, 8),
                                           ("staged224_gray192_J4_L8", 192, 192, 4, 8),
                                           ("staged384_gray256_J6_L7", 256, 256, 6, 7)])
def test_staged_general_geometries_chunking_and_parity(name, M, N, J, L):
    """Staged planes outside the square compiled-family route: rectangular (288 x 160 padded, row
    and column passes of different lengths, 144 x 80 level 1 with a runtime-length row pass),
    a padded size without a compiled staged FFT (224^2: generic DFT passes, 12 x 12 output maps)
    and odd L (unpaired last path in the all-paths s = 2 fold).  Golden parity at several batch
    positions, chunking invariance."""
    d, x = golden(name)
    ref = d["S"][0]
    rng = np.random.default_rng(5)
    xs = rng.integers(0, 256, (4, M, N), dtype=np.uint8).astype(np.float32) / 255
    pos = [0, 3]
    for i in pos:
        xs[i] = x[0]
    plan = _lib.Plan(M, N, J, L)
    xt = torch.from_numpy(xs).cuda()
    full = forward(plan, xt)
    small = forward(plan, xt, ws_planes=3)        # 2 chunks: 3 + 1 planes
    assert torch.equal(full, small), "chunked staged run differs"
    for i in pos:
        assert_parity(full[i].cpu().numpy()[None], ref[None], TOL, f"{name} @ {i}")
    assert torch.isfinite(full).all()


def test_staged_tall_plane_against_oracle():
    """The transposed orientation of the rectangular case (160 x 288 padded: row passes of 288
    points, column passes of 160), order 2, checked against the oracle directly."""
    x = np.random.default_rng(6).integers(0, 256, (1, 128, 256), dtype=np.uint8).astype(np.float32) / 255
    ref = kr.Scattering2D(J=4, shape=(128, 256), L=4)(x)
    got = NpS(J=4, shape=(128, 256), L=4)(x)
    assert got.shape == ref.shape == (1, 1 + 4 * 4 + 16 * 6, 8, 16)
    assert_parity(got, ref, TOL, "staged 128x256")


@pytest.mark.parametrize("M,N,J,L", [(200, 200, 3, 4),     # 216^2 padded, 25 x 25 maps
                                     (640, 600, 2, 2)])    # 648 x 608, 160 x 150 maps (taps in L2)
def test_staged_wide_output_maps_against_oracle(M, N, J, L):
    """Output maps wider than the LDS-resident low-pass (oM > 8): the staged column pass runs its
    outputs in groups of 16, reading the tap matrix from L2 when it does not fit beside the tile."""
    x = np.random.default_rng(7).integers(0, 256, (1, M, N), dtype=np.uint8).astype(np.float32) / 255
    ref = kr.Scattering2D(J=J, shape=(M, N), L=L)(x)
    got = NpS(J=J, shape=(M, N), L=L)(x)
    assert got.shape == ref.shape
    assert_parity(got, ref, TOL, f"staged {M}x{N} J={J}")


@pytest.mark.parametrize("M,J,L", [(224, 5, 4),     # 288^2 padded: 144^2 staged paths, 7 x 7 maps
                                   (256, 5, 3)])    # 320^2 padded: 160^2 staged paths, 8 x 8, odd L
def test_staged_order2_path_sizes_against_oracle(M, J, L):
    """Staged s = 2 order-2 levels at the compiled staged path sizes besides c5's 192^2 (goldens
    above): 144^2 and 160^2 paths of 288^2 / 320^2 padded planes, against the oracle."""
    x = np.random.default_rng(8).integers(0, 256, (2, M, M), dtype=np.uint8).astype(np.float32) / 255
    ref = kr.Scattering2D(J=J, shape=(M, M), L=L)(x)
    got = NpS(J=J, shape=(M, M), L=L)(x)
    assert got.shape == ref.shape
    assert_parity(got, ref, TOL, f"fused order-2 {M}^2 J={J} L={L}")


def test_staged_lines_beyond_lds_tiles_are_unsupported():
    with pytest.raises(_lib.WSTError) as e:
        _lib.Plan(2048, 2048, 2, 2)                # 2056^2 padded: 2056-point lines
    assert e.value.code == _lib.WST_ERR_UNSUPPORTED
    # the limit printed is the largest line the row / column tiles (and taps) actually admit
    assert "at most 1203 points" in str(e.value), str(e.value)


def test_staged_final_map_beyond_lds_is_unsupported():
    # 1000^2 J=2: 1008-point staged lines fit the tiles, but the 250 x 250 output maps (250 KB)
    # exceed k_big_final's LDS map: rejected at plan creation, not at wst_forward
    with pytest.raises(_lib.WSTError) as e:
        _lib.Plan(1000, 1000, 2, 8)
    assert e.value.code == _lib.WST_ERR_UNSUPPORTED
    assert "250x250 output maps" in str(e.value), str(e.value)
