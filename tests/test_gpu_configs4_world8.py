"""BASELINE configs[4] at FULL size through the multi-rank path: 8 gloo ranks sharing cuda:0 (the
exchanges staged through host memory by collective.TorchCollective; RCCL refuses two ranks on one
device, so the driver's 8-GPU node is where RCCL itself runs).

* (i)  2^26 four-step DFT split over 8 ranks, both output layouts (one and two all_to_alls): every
       rank's block equals the world-1 eon_fourstep_dft_dev output (itself checked against the
       single-network DFT in the same run).
* (ii) 2^24-term MSM over the alpha = 12345 SRS split by point range over 8 ranks
       (eon_msm_sharded_dev): the result equals [f(alpha)] G, f(alpha) from the C oracle's Horner.
"""

import pytest

from _launch import run_world

pytestmark = pytest.mark.gpu


def test_fourstep_dft_2_26_world8():
    res = run_world("fourstep_full", 8, timeout=600, extra_env={"EON_T_LOG_N": "26"})
    assert all(r["ok"] for r in res), [r["why"] for r in res]


def test_msm_2_24_world8_kzg_identity():
    res = run_world("msmshard_full", 8, timeout=600, extra_env={"EON_T_LOG_N": "24"})
    assert all(r["ok"] for r in res), [r["why"] for r in res]
