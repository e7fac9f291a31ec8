"""Frontend argument checking (kymatio 0.3.0 behaviour) and the no-CPU-fallback contract."""
import numpy as np
import pytest
import torch

import wst_amd
from wst_amd import features
from wst_amd.numpy import Scattering2D as NpS
from wst_amd.torch import Scattering2D as ThS


def test_build_errors():
    with pytest.raises(RuntimeError, match="2\\^J"):
        NpS(J=7, shape=(64, 64))
    with pytest.raises(RuntimeError):
        ThS(J=2, shape=(64, 64), max_order=3)


def test_entry_dispatch():
    assert isinstance(wst_amd.Scattering2D(J=2, shape=(32, 32), frontend="numpy"), NpS)
    assert isinstance(wst_amd.Scattering2D(J=2, shape=(32, 32), frontend="torch"), ThS)
    with pytest.raises(RuntimeError):
        wst_amd.Scattering2D(J=2, shape=(32, 32), frontend="jax")


def test_input_checks_precede_gpu():
    s = NpS(J=2, shape=(32, 32), L=4)
    with pytest.raises(TypeError):
        s(torch.zeros(32, 32))
    with pytest.raises(TypeError):
        s(np.zeros((32, 32), np.complex64))
    with pytest.raises(RuntimeError):
        s(np.zeros(32, np.float32))
    with pytest.raises(RuntimeError):
        s(np.zeros((30, 32), np.float32))
    t = ThS(J=2, shape=(32, 32), L=4)
    with pytest.raises(TypeError):
        t(np.zeros((32, 32), np.float32))
    with pytest.raises(RuntimeError):
        t(torch.zeros(32, 64)[:, ::2])          # non-contiguous
    bad = NpS(J=2, shape=(32, 32), L=4, out_type="dict")
    with pytest.raises(RuntimeError):
        bad(np.zeros((32, 32), np.float32))
    pp = NpS(J=2, shape=(32, 32), L=4, pre_pad=True)
    with pytest.raises(RuntimeError):
        pp(np.zeros((32, 32), np.float32))     # must be padded size (40, 40)


@pytest.mark.skipif(torch.cuda.is_available(), reason="CPU-only contract")
def test_no_cpu_fallback():
    with pytest.raises(RuntimeError, match="no ROCm GPU"):
        NpS(J=2, shape=(32, 32), L=4)(np.zeros((32, 32), np.float32))
    with pytest.raises(RuntimeError, match="no ROCm GPU"):
        ThS(J=2, shape=(32, 32), L=4)(torch.zeros(32, 32))


def test_feature_names():
    names = features.get_feature_names(2, 8)
    assert len(names) == 486 and names[0] == "R_wst_mean_0" and names[81] == "R_wst_std_0"
    assert names[162] == "G_wst_mean_0" and names[-1] == "B_wst_std_80"
    assert len(features.get_feature_names(4, 8)) == 3 * 2 * 417


def test_meta_order_matches_oracle_index():
    from oracle import kymatio_ref as kr
    s = NpS(J=3, shape=(32, 32), L=6)
    meta = s.meta()
    assert len(meta) == s.K == 127
    for k, m in enumerate(meta):
        if len(m["j"]) == 1:
            assert k == kr.coefficient_index(3, 6, m["j"][0], m["theta"][0])
        elif len(m["j"]) == 2:
            assert k == kr.coefficient_index(3, 6, m["j"][0], m["theta"][0], m["j"][1], m["theta"][1])


def test_feature_names_match_reference_artifacts():
    # layout pin: the 486 / 540 names every WST / hybrid experiment saved
    # (train_and_save_model.py:400-427), copied as data into tests/golden/ref_feature_names.json
    import json
    import os
    from conftest import GOLDEN
    ref = json.load(open(os.path.join(GOLDEN, "ref_feature_names.json")))
    assert features.get_feature_names(2, 8) == ref["wst"]
    assert ref["hybrid"][54:] == ref["wst"]
