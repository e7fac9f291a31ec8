"""CPU tests of bench.py's host logic and of the c3 patch generator's host restatement.

* ``bench.py --gpus 2`` started without WORLD_SIZE launches itself as two ranks through
  torch.distributed.run (``--launch-check``: the rank plumbing alone, gloo, no GPU).
* Kernel naming of the timing slots (c5's HBM-staged slots are composites).
* oracle/patchgen.py's Philox4x32-10 against the Random123 known-answer vectors (the device
  generator k_patch_generate runs the same round function; tests/test_gpu_workloads.py pins the
  two bit-exactly).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import patchgen  # noqa: E402


def test_gpus_2_launches_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    chk = lines[0]["launch_check"]
    assert chk == {"world": 2, "gpus": 2, "rank_sum": 3.0, "ok": True}


def test_rocprof_names():
    assert bench.rocprof_name("k_o2_j1=0", 96, 96, 4) == "k_o2<3, 3, 136"
    assert bench.rocprof_name("k_o1_j1=1", 136, 136, 2) == "k_o1<17, 17, 136"
    assert bench.rocprof_name("k_prep", 96, 96, 4) == "k_prep<3, 3"
    # c5: P = 384, levels 384 / 192 staged; k_o2 at j1 = 2 (96^2) is the family-3 resident kernel
    assert bench.staged_levels(384, 384, 6) == 2
    assert bench.rocprof_name("k_o2_j1=2", 384, 384, 6) == "k_o2<3, 3, 136"
    assert "k_o2<3, 3, 136, 1, 1" in bench.rocprof_name("k_o2_j1=0", 384, 384, 6)
    assert "k_big_rows<192, 1>" in bench.rocprof_name("k_o1_j1=1", 384, 384, 6)


def test_staged_slot_traffic_from_dispatch_sequence():
    # c5 (384^2, J=6, L=12, square family 3: rb = nst = 2): one chunk = 39 staged launches
    # (S0 + Xhat 4; per staged j1: order 1 3 + U1hat half rows 1; j1 = 0's 192^2 order 2 24 + final
    # + HG k_o2; j1 = 1's HG k_o2)
    seq = bench.staged_sequence(384, 384, 6, 12, 2)
    assert len(seq) == 4 + 4 + (2 * 12 + 1 + 1) + 4 + 1
    assert seq[-1] == ("k_o2_j1=1", "k_o2<3, 3, 136, 1, 1>")
    # a recorded run: two chunks, each followed by resident kernels, one byte count per launch
    disp = []
    for c in range(2):
        disp += [[k, 10 if sl == "k_o2_j1=0" else 1] for sl, k in seq]
        disp += [["k_o1<3, 3, 136, 1>", 7], ["k_o2<3, 3, 136, 1, 0>", 7]]
    summ = {"dispatch_seq": disp}
    assert bench.slot_traffic(summ, seq, "k_o2_j1=0") == 10 * (2 * 12 + 2)
    assert bench.slot_traffic(summ, seq, "k_prep") == 4
    assert bench.slot_traffic({"dispatch_seq": disp[5:]}, seq, "k_prep") == 4   # first chunk cut
    assert bench.slot_traffic({}, seq, "k_prep") is None
    # non-square / uncompiled sizes: every order-2 level staged, runtime-length passes named <0, ...>
    seq2 = bench.staged_sequence(288, 160, 4, 8, 4)
    assert ("k_o2_j1=0", "k_big_rows<0, true>") in seq2            # 80-point rows at level 1
    assert not any(k.startswith("k_o2<") for _, k in seq2)


def test_alg_flops_split_sums_to_the_cascade():
    # c2: 115.4 MFLOP per RGB patch
    f = bench.alg_flops_per_plane(96, 96, 4, 8)
    assert abs(3 * sum(f.values()) / 1e6 - 115.4) < 0.1


@pytest.mark.parametrize("ctr,key,expect", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox_known_answers(ctr, key, expect):
    got = patchgen.philox4x32_10(*ctr, *key)
    assert tuple(int(v) for v in got) == expect


def test_patchgen_is_keyed_by_global_index():
    a = patchgen.generate_patches_u8(1, 1000, 6, 3, 8, 8)
    b = np.concatenate([patchgen.generate_patches_u8(1, 1000, 2, 3, 8, 8),
                        patchgen.generate_patches_u8(1, 1002, 4, 3, 8, 8)])
    np.testing.assert_array_equal(a, b)
    assert not np.array_equal(a[0], a[1])
    c = patchgen.generate_patches_u8(2, 1000, 6, 3, 8, 8)
    assert not np.array_equal(a, c)
    # uniform bytes: mean ~127.5
    big = patchgen.generate_patches_u8(1, 0, 64, 3, 64, 64)
    assert abs(big.mean() - 127.5) < 1.0


def test_pmc_traffic_is_looked_up_per_config(tmp_path, monkeypatch):
    # c5's LDS-resident levels instantiate the same k_o2<3, 3, 136, ...> as c2: a c5 PMC file must
    # never supply c2's roofline.traffic (and vice versa)
    assert bench.pmc_file_config("pmc_r01s12.json") == "c2"
    assert bench.pmc_file_config("pmc_r02s4_c5.json") == "c5"
    assert bench.pmc_file_config("pmc_r02s4_f3.json") == "f3"
    prof = tmp_path / "profiles"
    prof.mkdir()
    name = "k_o2<3, 3, 136, 1, 0>"
    for fname, v in [("pmc_x_c2.json", 111), ("pmc_x_c5.json", 555)]:
        (prof / fname).write_text(json.dumps({"src_sha": "s", "hbm_bytes_per_launch": {name: v}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_traffic("s", "k_o2<3, 3, 136", "c2") == 111
    assert bench.pmc_traffic("s", "k_o2<3, 3, 136", "c3") == 111
    assert bench.pmc_traffic("s", "k_o2<3, 3, 136", "c5") == 555
    assert bench.pmc_traffic("s", "k_o2<3, 3, 136", "f3") is None
    assert bench.pmc_traffic("other", "k_o2<3, 3, 136", "c2") is None
