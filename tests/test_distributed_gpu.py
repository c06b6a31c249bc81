"""Lane-sharded prove through the product path (HIP kernels) with two gloo ranks sharing cuda:0:
every rank's proof must equal the unsharded prove bit for bit."""

import pytest

from _launch import run_world

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,log_n,vl", [(2, 5, 4), (4, 4, 8)])
def test_sharded_prove_matches_single(world, log_n, vl):
    res = run_world("gpu", world, timeout=900, extra_env={"EON_T_LOG_N": str(log_n), "EON_T_VL": str(vl)})
    assert all(r["ok"] for r in res), [r["why"] for r in res]


@pytest.mark.parametrize("world,log_n,vl", [(2, 5, 4), (4, 3, 8), (2, 17, 2), (8, 17, 8)])
def test_native_sharded_prove_matches_single(world, log_n, vl):
    """The C++ driver's lane-sharded prove (torch.distributed eon_collective) == its unsharded
    prove == the Python prover.  (8, 17, 8) is the driver's 8-GPU scaling configuration of the
    headline proof (one lane per rank of the VECTOR_LEN-8 2^17 trace), here with gloo ranks
    sharing one GPU."""
    res = run_world("native", world, timeout=900, extra_env={"EON_T_LOG_N": str(log_n), "EON_T_VL": str(vl)})
    assert all(r["ok"] for r in res), [r["why"] for r in res]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_fourstep_dft_matches_oracle(world):
    """eon_fourstep_dft_dev over a TorchCollective (gloo ranks sharing cuda:0), both layouts."""
    res = run_world("fourstep", world, timeout=900)
    assert all(r["ok"] for r in res), [r["why"] for r in res]


@pytest.mark.parametrize("world", [1, 3, 8])
def test_sharded_msm_matches_full(world):
    """eon_msm_sharded_dev: per-rank Pippenger + all-gather of partials + EC sum == the full MSM."""
    res = run_world("msmshard", world, timeout=900)
    assert all(r["ok"] for r in res), [r["why"] for r in res]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_opening_bases(world):
    """Opening bases split by rows over the ranks (two all-gathers) == each rank's own, at 2^17
    rows (world 3: uneven slices)."""
    res = run_world("openshard", world, timeout=900)
    assert all(r["ok"] for r in res), [r["why"] for r in res]


@pytest.mark.parametrize("mode,env", [("native", {"EON_T_LOG_N": "5", "EON_T_VL": "4"}), ("fourstep", {}),
                                      ("msmshard", {}), ("openshard", {})])
def test_rccl_process_group_world1(mode, env):
    """The same exchanges over torch.distributed's nccl backend (RCCL, device buffers), the
    backend bench.py runs at N > 1 GPUs: all_gather_into_tensor / all_to_all_single through
    TorchCollective.  RCCL takes one rank per GPU, so one box runs world 1; the N-rank exchange
    layouts are the gloo tests above."""
    res = run_world(mode, 1, timeout=900, extra_env=dict(env, EON_T_BACKEND="nccl"))
    assert all(r["ok"] for r in res), [r["why"] for r in res]


def test_rccl_collective_info_world1():
    """The driver's own RCCL communicator at world 1 reports itself (ncclCommCount 1, user rank 0,
    device 0, that device's PCI bus id), and bench.py's per-rank record of the same process carries
    those fields beside torch's own PCI address of the device -- the evidence an N-GPU line holds
    for every rank (bench.py rank_evidence)."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    code = (
        "import json, sys, torch; sys.path.insert(0, %r)\n"
        "torch.cuda.set_device(0)\n"
        "import bench\n"
        "from plonky3_eon_amd.native import RcclCollective\n"
        "c = RcclCollective(0, 1)\n"
        "class W: pass\n"
        "w = W(); w.coll = c; w.collective_kind = 'rccl'\n"
        "w.throughput = lambda world, ms: ({'stage_ms': {'x': 1.0}}, None)\n"
        "rec = bench.rank_evidence(w, 0, 0, torch.device('cuda', 0), 0.5, 5, 1)\n"
        "c.close()\n"
        "print(json.dumps(rec))\n" % str(root))
    out = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["nccl_comm_count"] == 1 and rec["nccl_user_rank"] == 0 and rec["nccl_cu_device"] == 0, rec
    assert rec["nccl_pci_bus_id"].lower() == rec["pci_bus_id"].lower(), rec  # RCCL's device = torch's
    assert rec["collective"] == "rccl" and rec["ms_per_step"] == 100.0
    assert rec["stage_ms"] == {"x": 1.0}
