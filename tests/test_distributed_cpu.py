"""Lane-sharded prove (plonky3_eon_amd/distributed.py) on CPU: world_size-2 gloo
ranks exchange oracle-computed partial quotients through the product's collective helpers."""

import pytest

from oracle import pyoracle as O
from plonky3_eon_amd import _lib
from plonky3_eon_amd import distributed as D

from _launch import run_world


def test_lane_ranges_partition():
    for world in (1, 2, 4, 8):
        got = [D.lane_range(r, world, 8) for r in range(world)]
        assert got[0][0] == 0 and got[-1][1] == 8
        assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
    with pytest.raises(_lib.EonError):
        D.lane_range(0, 3, 8)
    with pytest.raises(_lib.EonError):
        D.lane_range(2, 2, 8)


def test_lane_weights():
    a = 0x1234567890ABCDEF
    assert D.lane_weights(a, 8, 1, 160) == [1]
    w = D.lane_weights(a, 8, 4, 160)
    assert w[-1] == 1
    assert w[0] == pow(a, 160 * 6, O.P)
    assert w[1] == pow(a, 160 * 4, O.P)


def test_sharded_quotient_gloo_world2():
    res = run_world("cpu", 2, timeout=600)
    assert all(r["ok"] for r in res), [r["why"] for r in res]


def test_sharded_quotient_gloo_world4():
    res = run_world("cpu", 4, timeout=600)
    assert all(r["ok"] for r in res), [r["why"] for r in res]


@pytest.mark.parametrize("world", [1, 2, 4])
def test_fourstep_exchange_gloo(world):
    res = run_world("a2a", world, timeout=600)
    assert all(r["ok"] for r in res), [r["why"] for r in res]


def test_shard_range_partition():
    for n in (1, 7, 4096, 4099):
        for world in (1, 2, 3, 8):
            r = [D.shard_range(n, g, world) for g in range(world)]
            assert r[0][0] == 0 and r[-1][1] == n and all(a[1] == b[0] for a, b in zip(r, r[1:]))


@pytest.mark.parametrize("fail", ["none", "id", "init1"])
def test_rccl_init_outcome_agreed_gloo(fail):
    """native.RcclCollective ends the same way on every rank: a failed unique id on
    rank 0 or a failed communicator init on rank 1 makes every rank raise RcclInitError (so
    bench.py's fallback to torch.distributed is taken by all ranks together), and no rank waits in
    a broadcast rank 0 skipped.  Fake driver library, gloo world 3."""
    res = run_world("rcclagree", 3, timeout=300, extra_env={"EON_T_FAIL": fail})
    assert all(r["ok"] for r in res), [r["why"] for r in res]
