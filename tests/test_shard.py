"""Utterance sharding over ranks: LPT plan properties, and world_size-2 gloo runs whose
gathered codes equal the single-process result bit-exactly (CPU: oracle generator; GPU: HIP path)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from tests.helpers import load_golden, synthetic_weights
from zonos_vibes_amd.config import ZonosConfig
from zonos_vibes_amd.shard import estimated_frames, gather_codes, generate_sharded, lpt_assign

N_UTT = 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs():
    t, meta = load_golden("tiny_trajectories")
    cfg = ZonosConfig.from_dict(meta["cfg"])
    g = torch.Generator().manual_seed(7)
    d = cfg.backbone.d_model
    conds = [torch.randn(2, 6 + 2 * i, d, generator=g).to(torch.bfloat16) for i in range(N_UTT)]
    mnt = [10, 4, 14, 7, 12]
    return cfg, conds, mnt


class OracleBatch:
    """generate_batch() over the CPU oracle, one utterance at a time (test stand-in for Zonos)."""

    def __init__(self, cfg):
        from oracle.zonos_cpu import OracleZonos
        self.m = OracleZonos(cfg, synthetic_weights(cfg, zero_eos=True))

    def generate_batch(self, conds, prefixes=None, max_new_tokens=10, cfg_scale=2.0, sampling_params=None,
                       seeds=None, **kw):
        return [self.m.generate(c, p, max_new_tokens=n, cfg_scale=cfg_scale, sampling_params=sampling_params)
                for c, p, n in zip(conds, prefixes, max_new_tokens)]


def test_lpt_partitions_and_balances():
    costs = [5, 9, 1, 9, 3, 7, 7, 2, 8]
    for world in (1, 2, 3, 4, 8, 12):
        parts = lpt_assign(costs, world)
        flat = sorted(i for p in parts for i in p)
        assert flat == list(range(len(costs)))
        assert parts == lpt_assign(costs, world)  # deterministic: every rank derives the same plan
        loads = [sum(costs[i] for i in p) for p in parts]
        assert max(loads) <= sum(costs) / world + max(costs)  # LPT bound
    assert lpt_assign([], 2) == [[], []]
    with pytest.raises(ValueError):
        lpt_assign([1], 0)


def test_estimated_frames_counts_prefix_and_conditioning():
    c = torch.zeros(2, 10, 4)
    p = torch.zeros(1, 9, 3, dtype=torch.long)
    assert estimated_frames([c, c], [None, p], [100, 100]) == [100 + 8 + 11, 100 + 8 + 14]


def test_single_rank_gather_is_identity():
    a, b = torch.ones(1, 9, 3, dtype=torch.long), torch.zeros(1, 9, 2, dtype=torch.long)
    out = gather_codes([a, b], [1, 0], 2)
    assert out[0] is b and out[1] is a


def _cpu_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        cfg, conds, mnt = _inputs()
        mine, local, gathered = generate_sharded(OracleBatch(cfg), conds, max_new_tokens=mnt,
                                                 sampling_params=dict(temperature=0.0))
        torch.save({"mine": mine, "gathered": gathered}, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_equal_single_process(tmp_path):
    port = _free_port()
    mp.spawn(_cpu_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert r1["gathered"] is None
    assert sorted(r0["mine"] + r1["mine"]) == list(range(N_UTT)) and r0["mine"] and r1["mine"]
    torch.set_num_threads(1)
    cfg, conds, mnt = _inputs()
    ref = OracleBatch(cfg).generate_batch(conds, [None] * N_UTT, mnt, sampling_params=dict(temperature=0.0))
    for i in range(N_UTT):
        assert torch.equal(r0["gathered"][i], ref[i]), i


def _gpu_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from zonos_vibes_amd.model import Zonos
        cfg, conds, mnt = _inputs()
        m = Zonos.synthetic(cfg, "cuda:0", zero_eos=True, max_seqlen=64, max_prefill=32)
        mine, local, gathered = generate_sharded(m, [c.to("cuda:0") for c in conds], max_new_tokens=mnt,
                                                 sampling_params=dict(temperature=0.0))
        torch.save({"mine": mine, "gathered": gathered}, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_two_ranks_equal_single_process(tmp_path):
    """Two ranks (both on cuda:0, gloo) vs generate() per utterance in this process: bit-identical."""
    from zonos_vibes_amd.model import Zonos
    port = _free_port()
    mp.spawn(_gpu_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    got = torch.load(tmp_path / "r0.pt", weights_only=True)["gathered"]
    cfg, conds, mnt = _inputs()
    m = Zonos.synthetic(cfg, "cuda:0", zero_eos=True, max_seqlen=64, max_prefill=32)
    for i in range(N_UTT):
        ref = m.generate(conds[i].to("cuda:0"), max_new_tokens=mnt[i], sampling_params=dict(temperature=0.0),
                         progress_bar=False).cpu()
        assert torch.equal(got[i], ref), i


def _rccl_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from zonos_vibes_amd.shard import _gather_collective
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(3)
        local = [torch.randint(0, 1026, (1, 9, t), generator=g) for t in (7, 1, 33)]
        got = _gather_collective(local, [2, 0, 1], 3, 0, None, torch.device("cuda", 0), rank, world)
        torch.save({"local": local, "got": [c.cpu() for c in got]}, os.path.join(out_dir, "rccl.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_int16_gather_path_on_one_gpu(tmp_path):
    """gather_codes' collective path on RCCL (backend "nccl") with one rank on cuda:0: the size headers and the
    2-byte code payload go through RCCL all_gathers on the device and come back in global utterance order (the
    multi-rank path the 8-GPU bench would take; a one-GPU box cannot run two RCCL ranks). This test found that
    RCCL has no int16 all_gather: the payload now travels as a bfloat16 view of the int16 codes."""
    port = _free_port()
    mp.spawn(_rccl_worker, args=(1, port, str(tmp_path)), nprocs=1, join=True)
    r = torch.load(tmp_path / "rccl.pt", weights_only=True)
    local, got = r["local"], r["got"]
    assert [tuple(c.shape) for c in got] == [(1, 9, 1), (1, 9, 33), (1, 9, 7)]
    assert torch.equal(got[2], local[0]) and torch.equal(got[0], local[1]) and torch.equal(got[1], local[2])
