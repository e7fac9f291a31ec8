"""GPU parity tests: the HIP path (through the C ABI / the kymatio-compatible frontends) against
the float64 oracle and its committed golden fixtures.

Tolerance (written here, per SURVEY.md §8(c) / BASELINE north_star): per coefficient index k,
max|S_gpu - S_ref|[k] / max|S_ref[k]| <= 1e-5 (parity.TOL).
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden
from oracle import kymatio_ref as kr
from parity import TOL, assert_parity, per_coef_error

import wst_amd
from wst_amd import _lib, features
from wst_amd.numpy import Scattering2D as NpS
from wst_amd.torch import Scattering2D as ThS

pytestmark = pytest.mark.gpu
PHI0 = np.pi / 3.1415

with open(os.path.join(GOLDEN, "manifest.json")) as _fh:
    MANIFEST = json.load(_fh)


def golden_input(name):
    d = load_golden(name)
    return d, d["x_u8"].astype(np.float32) / 255


def rgb(seed, shape):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8).astype(np.float32) / 255


def test_gpu_present_and_library_loaded():
    assert torch.cuda.is_available(), "GPU tests need a ROCm GPU"
    lib = _lib.load()
    assert lib.wst_abi_version() == _lib.ABI_VERSION


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_golden_parity_numpy_frontend(name):
    m = MANIFEST[name]
    d, x = golden_input(name)
    s = NpS(J=m["J"], shape=(m["M"], m["N"]), L=m["L"], max_order=m["max_order"])
    try:
        S = s(x)
    except _lib.WSTError as e:
        if e.code == _lib.WST_ERR_UNSUPPORTED:
            pytest.skip(f"{name}: not yet covered by the HIP path: {e}")
        raise
    assert S.shape == d["S"].shape and S.dtype == np.float64   # kymatio.numpy returns float64
    assert_parity(S, d["S"], TOL, name)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_numpy_frontend_dtype_contract(dtype):
    # kymatio.numpy multiplies by float64 filters: float32 input (train_and_save_model.py:51-56,368)
    # and float64 input both come back float64; the torch frontend keeps float32 on the device
    d, x = golden_input("c2_rgb64_J4_L8")
    s = NpS(J=4, shape=(64, 64), L=8)
    S = s(x.astype(dtype))
    assert S.dtype == np.float64 and S.shape == d["S"].shape
    assert_parity(S, d["S"], TOL, "c2 dtype " + np.dtype(dtype).name)
    F = s.pooled(x.astype(dtype))
    assert F.dtype == np.float64 and F.shape == (3, 2 * 417)


@pytest.mark.parametrize("name", ["c2_rgb64_J4_L8", "c1_rgb64_J2_L8"])
def test_golden_parity_torch_frontend_on_device(name):
    m = MANIFEST[name]
    d, x = golden_input(name)
    s = ThS(J=m["J"], shape=(m["M"], m["N"]), L=m["L"])
    xt = torch.from_numpy(x).cuda()
    S = s(xt)
    assert S.is_cuda and S.dtype == torch.float32
    assert_parity(S.cpu().numpy(), d["S"], TOL, name)


def test_torch_cpu_tensor_like_inference_py():
    # inference.py:250-257: (1,1,H,W) contiguous float32 CPU tensor under no_grad -> squeeze
    d, x = golden_input("c1_rgb64_J2_L8")
    S = ThS(J=2, shape=(64, 64), L=8)
    with torch.no_grad():
        out = S(torch.from_numpy(x[1]).unsqueeze(0).unsqueeze(0).contiguous())
    assert out.device.type == "cpu" and tuple(out.shape) == (1, 1, 81, 16, 16)
    assert_parity(out.squeeze(0).squeeze(0).numpy()[None], d["S"][1:2], TOL)


def test_training_and_inference_feature_layouts():
    d, x = golden_input("c1_rgb64_J2_L8")
    absmax = d["S_absmax"].astype(np.float64)            # (C, K)
    f = features.extract_wst_features(x, J=2, L=8)
    assert f.shape == (486,) and f.dtype == np.float64
    ref = d["features_train"].reshape(3, 2, 81)
    got = f.reshape(3, 2, 81)
    assert np.all(np.abs(got[:, 0] - ref[:, 0]) <= TOL * absmax)        # means
    assert np.all(np.abs(got[:, 1] - ref[:, 1]) <= 2 * TOL * absmax)    # stds (|d std| <= 2 max|dS|)
    g = features.extract_wst_features_interleaved(x, J=2, L=8)
    np.testing.assert_array_equal(g.reshape(3, 81, 2), np.moveaxis(got, 1, 2))


@pytest.mark.parametrize("M,J", [(64, 4),     # 4 x 4 maps: one thread per map
                                 (64, 2),     # 16 x 16: one wave per map
                                 (128, 2)])   # 32 x 32: the reference's training geometry
def test_pooled_equals_pooling_of_full_output(M, J):
    x = rgb(5, (16 if M == 64 else 4, 3, M, M))
    s = ThS(J=J, shape=(M, M), L=8)
    xt = torch.from_numpy(x).cuda()
    S = s(xt).double()
    P = s.pooled(xt).double()
    K = s.K
    mean = S.mean(dim=(-2, -1))
    std = S.std(dim=(-2, -1), unbiased=False)
    scale = S.abs().amax(dim=(0, 1, 3, 4))
    assert torch.all((P[..., :K] - mean).abs() <= 1e-6 * scale)
    assert torch.all((P[..., K:] - std).abs() <= 1e-6 * scale)


def test_batch_position_invariance_and_determinism():
    x = rgb(6, (37, 64, 64))
    x[20] = x[3]
    s = ThS(J=4, shape=(64, 64), L=8)
    xt = torch.from_numpy(x).cuda()
    a = s(xt)
    b = s(xt)
    assert torch.equal(a, b), "two runs differ"
    assert torch.equal(a[20], a[3]), "result depends on batch position"


def test_chunked_workspace_bitwise_equal():
    x = torch.from_numpy(rgb(7, (23, 64, 64))).cuda()
    plan = _lib.Plan(64, 64, 4, 8)
    out_full = torch.empty((23, plan.K, plan.Mo, plan.No), device="cuda")
    out_chunk = torch.empty_like(out_full)
    ws_full = torch.empty(plan.workspace_bytes(23), dtype=torch.uint8, device="cuda")
    ws_small = torch.empty(plan.workspace_bytes(5), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    plan.forward(x.data_ptr(), 23, out_full.data_ptr(), False, ws_full.data_ptr(), ws_full.numel(), st)
    plan.forward(x.data_ptr(), 23, out_chunk.data_ptr(), False, ws_small.data_ptr(), ws_small.numel(), st)
    # internal workspace path (NULL workspace)
    out_int = torch.empty_like(out_full)
    plan.forward(x.data_ptr(), 23, out_int.data_ptr(), False, 0, 0, st)
    torch.cuda.synchronize()
    assert torch.equal(out_full, out_chunk) and torch.equal(out_full, out_int)


def test_empty_batch_and_batch_shapes():
    s = ThS(J=2, shape=(32, 32), L=4)
    out = s(torch.zeros((0, 32, 32), device="cuda"))
    assert tuple(out.shape) == (0, s.K, 8, 8)
    x = torch.from_numpy(rgb(8, (2, 3, 32, 32))).cuda()
    out = s(x)
    assert tuple(out.shape) == (2, 3, s.K, 8, 8)
    np.testing.assert_array_equal(out[1, 2].cpu().numpy(), s(x[1, 2].contiguous()).cpu().numpy())


def test_pre_pad_equals_internal_padding():
    M, J = 32, 2
    s = NpS(J=J, shape=(M, M), L=4)
    sp = NpS(J=J, shape=(M, M), L=4, pre_pad=True)
    x = rgb(9, (3, M, M))
    p = kr.compute_padding(M, M, J)[0] - M
    xp = np.pad(x, ((0, 0), (p // 2, (p + 1) // 2), (p // 2, (p + 1) // 2)), mode="reflect")
    np.testing.assert_allclose(sp(xp), s(x), rtol=0, atol=1e-6)


def test_out_type_list():
    s = NpS(J=2, shape=(32, 32), L=4, out_type="list")
    x = rgb(10, (32, 32))
    lst = s(x)
    arr = NpS(J=2, shape=(32, 32), L=4)(x)
    assert len(lst) == arr.shape[0]
    assert lst[0]["j"] == () and lst[1]["j"] == (0,) and lst[-1]["j"] == (0, 1)
    np.testing.assert_array_equal(lst[5]["coef"], arr[5])


def test_constant_image_known_answer():
    s = NpS(J=4, shape=(64, 64), L=8)
    S = s(np.full((2, 64, 64), 0.25, np.float32))
    np.testing.assert_allclose(S[:, 0], 0.25 * PHI0, rtol=2e-6)
    assert np.abs(S[:, 1:]).max() < 1e-6


def test_full_size_c2_properties_and_sampled_oracle():
    """BASELINE config 2 at its full size (1024 RGB patches = 3072 planes, J=4, L=8):
    size-independent properties over the whole batch + oracle parity on sampled planes."""
    B = 1024
    x = torch.from_numpy(rgb(11, (B, 3, 64, 64))).cuda()
    s = ThS(J=4, shape=(64, 64), L=8)
    S = s(x)
    assert tuple(S.shape) == (B, 3, 417, 4, 4)
    assert torch.isfinite(S).all()
    a, b = 0.5, 0.25
    S2 = s(a * x + b)
    # S0 affine; S1/S2 shift-invariant and positively homogeneous
    d0 = (S2[:, :, 0] - (a * S[:, :, 0] + PHI0 * b)).abs().max().item()
    assert d0 <= TOL * S2[:, :, 0].abs().max().item()
    Sd, S2d = S.double(), S2.double()
    scale = (a * Sd[:, :, 1:]).abs().amax(dim=(0, 1, 3, 4))
    err = ((S2d[:, :, 1:] - a * Sd[:, :, 1:]).abs().amax(dim=(0, 1, 3, 4)) / scale).max().item()
    assert err <= 2 * TOL, err
    # oracle on 6 sampled planes
    idx = [(0, 0), (17, 1), (255, 2), (511, 0), (777, 1), (1023, 2)]
    sc = kr.Scattering2D(J=4, shape=(64, 64), L=8)
    xs = np.stack([x[i, c].cpu().numpy() for i, c in idx])
    ref = sc(xs)
    got = np.stack([S[i, c].cpu().numpy() for i, c in idx])
    assert_parity(got, ref, TOL, "c2 sampled")


# Geometries whose SQ kernels run with compile-time level sizes for families other than the
# headline's 3 (wst_device.h unique_level), a family-1 plane (two sizes per class: runtime sizes),
# the families of common patch sizes (7, 11, 13, 15, 27) and a family-19 plane (generic DFT), each
# against the float64 oracle computed here.
@pytest.mark.parametrize("M,J,L", [(48, 4, 8),    # P = 80 (family 5): 80 / 40 / 20 compile-time
                                   (56, 3, 6),    # P = 72 (family 9): 72 / 36 / 18 compile-time
                                   (48, 3, 8),    # P = 64 (family 1): 64 and 128 share a class
                                   (40, 3, 8),    # P = 56 (family 7)
                                   (48, 2, 8),    # P = 56 (family 7): 16 x 16 maps (wide low-pass)
                                   (80, 2, 4),    # P = 88 (family 11)
                                   (96, 2, 4),    # P = 104 (family 13)
                                   (112, 2, 4),   # P = 120 (family 15)
                                   (100, 2, 4),   # P = 108 (family 27)
                                   (68, 2, 4)])   # P = 76 (family 19): generic DFT
def test_family_geometries_against_oracle(M, J, L):
    x = rgb(7 + M + J, (2, M, M))
    got = NpS(J=J, shape=(M, M), L=L)(x)
    ref = kr.Scattering2D(J=J, shape=(M, M), L=L)(x)
    assert_parity(got, ref, what=f"{M}x{M} J={J} L={L}")


def test_internal_workspace_streams_bounded_and_bitwise_equal():
    # per-stream internal workspaces are capped (LRU, evicted once their work is done);
    # every stream's result equals the caller-workspace result bit for bit
    d, x = golden_input("c2_rgb64_J4_L8")
    plan = _lib.Plan(64, 64, 4, 8)
    xt = torch.from_numpy(np.concatenate([x] * 4, 0)).cuda()
    B = xt.shape[0]
    ref = torch.empty((B, plan.K, plan.Mo, plan.No), device="cuda")
    ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device="cuda")
    plan.forward(xt.data_ptr(), B, ref.data_ptr(), False, ws.data_ptr(), ws.numel(),
                 torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(6)]
    outs = []
    for rep in range(2):
        for s in streams:
            o = torch.empty_like(ref)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                plan.forward(xt.data_ptr(), B, o.data_ptr(), False, 0, 0, s.cuda_stream)
            outs.append((s, o))
            n, nbytes = plan.internal_workspaces()
            assert 1 <= n <= 4, n
            assert nbytes <= 4 * plan.workspace_bytes(B)
    torch.cuda.synchronize()
    for _, o in outs:
        assert torch.equal(o, ref)
