"""The one-workgroup-per-slot greedy sampler (zmi_sample_step_greedy) against zmi_sample_step (mode 0, the
per-codebook workgroups pinned to the reference in test_gpu_kernels.py / test_gpu_fsm.py): from the same slot
state, logits and history, every output must be identical — tokens, the delayed frame write, the slot
counters, the next step's rows (kv row, position) and the fused embedding of the next input frame. Covers
CFG, exact logit ties (first index wins), EOS forcing and the stopping diagonal, penalty windows (0 = whole
history, negative, 2, 40), no penalty, inactive slots and the max-length tail."""
import ctypes

import pytest
import torch

from zonos_vibes_amd.engine import SamplingParams

pytestmark = pytest.mark.gpu
DEV = "cuda"
S, D, TCAP = 4, 256, 96


def _state(seed, params_list):
    from zonos_vibes_amd import _lib as L
    g = torch.Generator().manual_seed(seed)
    st = {k: torch.zeros(S, dtype=torch.int32) for k in ("active", "pos", "offset", "remaining", "stopping", "step",
                                                          "total_len")}
    delayed = torch.randint(0, 1026, (S, 9, TCAP), generator=g, dtype=torch.int32)
    for s in range(S):
        off = int(torch.randint(12, 60, (1,), generator=g))
        st["offset"][s] = off
        st["pos"][s] = off + 20
        st["remaining"][s] = [30, 9, 3, 1][s]
        st["stopping"][s] = s == 2
        st["step"][s] = off
        st["total_len"][s] = [TCAP - 4, TCAP - 4, TCAP - 4, off + 1][s]  # slot 3: frame past the total length
        st["active"][s] = s != 1 or seed % 2 == 0
        delayed[s, :, off + 1:] = -1  # the frame being written and later ones are unknown
        delayed[s, 5:, off + 1] = 7   # ... except the delay-pattern's already-known cells
    prm = b"".join(bytes(bytearray(p.to_c())) for p in params_list)
    logits = torch.randn(2 * S, 9, 1026, generator=g) * 3
    logits[:, :, 100] = logits[:, :, 101] = 50.0  # exact ties: the first index wins
    logits[0, 0, 1024] = 80.0                     # slot 0 codebook 0 picks EOS
    emb = (torch.randn(9, 1026, D, generator=g) * 0.1).to(torch.bfloat16)
    return st, delayed, prm, logits, emb, L


def _run(st, delayed, prm, logits, emb, L, greedy):
    lib, sp = L.lib(), torch.cuda.current_stream().cuda_stream
    st = {k: v.clone().to(DEV) for k, v in st.items()}
    delayed = delayed.clone().to(DEV)
    prm_t = torch.tensor(bytearray(prm), dtype=torch.uint8).to(DEV)
    sl = L.Slots(*(st[k].data_ptr() for k in ("active", "pos", "offset", "remaining", "stopping", "step")),
                 delayed.data_ptr(), prm_t.data_ptr(), st["total_len"].data_ptr(), TCAP, S)
    lg = logits.to(DEV)
    e = emb.to(DEV)
    nxt = torch.full((S, 9), -7, dtype=torch.int32, device=DEV)
    cnt = torch.zeros(S, dtype=torch.int32, device=DEV)
    x = torch.zeros(2 * S, D, dtype=torch.bfloat16, device=DEV)
    row_kv = torch.full((2 * S,), -3, dtype=torch.int32, device=DEV)
    row_pos = torch.full((2 * S,), -3, dtype=torch.int32, device=DEV)
    if greedy:
        L.check(lib.zmi_sample_step_greedy(ctypes.byref(sl), lg.data_ptr(), nxt.data_ptr(), 0, S, e.data_ptr(), D,
                                           x.data_ptr(), row_kv.data_ptr(), row_pos.data_ptr(), sp))
    else:
        L.check(lib.zmi_sample_step(ctypes.byref(sl), lg.data_ptr(), None, nxt.data_ptr(), cnt.data_ptr(), 0, 0, S,
                                    e.data_ptr(), D, x.data_ptr(), row_kv.data_ptr(), row_pos.data_ptr(), sp))
    torch.cuda.synchronize()
    return dict(next=nxt.cpu(), delayed=delayed.cpu(), x=x.cpu(), row_kv=row_kv.cpu(), row_pos=row_pos.cpu(),
                **{k: v.cpu() for k, v in st.items()})


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("pen", [(3.0, 2), (3.0, 0), (2.0, -5), (1.5, 40), (1.0, 2)])
def test_greedy_sampler_identical_to_codebook_workgroups(seed, pen):
    params = [SamplingParams(temperature=0.0, repetition_penalty=pen[0], repetition_penalty_window=pen[1],
                             cfg_scale=c) for c in (2.0, 1.0, 3.0, 2.0)]
    args = _state(seed, params)
    ref = _run(*args, greedy=False)
    got = _run(*args, greedy=True)
    for k in ref:
        if k == "next":  # inactive slots leave their tokens untouched in both; active ones must agree
            act = args[0]["active"].bool()
            assert torch.equal(got[k][act], ref[k][act]), k
        else:
            assert torch.equal(got[k], ref[k]), k
