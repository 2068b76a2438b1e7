"""The EOS state machine, the EOS/mask diagonal and the masked_scatter_ frame write of the HIP
sampler (zmi_sample_step), driven with the reference's own logits so the check is exact:
reference zonos/model.py:255-311 (EOS -> remaining = min(remaining, 9), forced mask/EOS diagonal,
`frame.masked_scatter_(frame == -1, next_token)` compaction, including the max-length tail where
the masked slots are a suffix and receive the tokens of the first codebooks)."""
import ctypes

import pytest
import torch

from tests.helpers import load_golden, synthetic_weights
from zonos_vibes_amd.config import ZonosConfig

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = ["greedy_maxlen", "greedy_prefix", "greedy_eos_0", "greedy_eos_1"]


@pytest.mark.parametrize("greedy_kernel", [False, True])
@pytest.mark.parametrize("tag", CASES)
def test_fsm_and_frame_write_match_reference(tag, greedy_kernel):
    """greedy_kernel: decode steps through zmi_sample_step_greedy (one workgroup per slot) instead of
    zmi_sample_step's per-codebook workgroups."""
    from oracle.zonos_cpu import OracleZonos
    from zonos_vibes_amd import _lib as L
    from zonos_vibes_amd.engine import SamplingParams
    t, meta = load_golden("tiny_trajectories")
    cfg = ZonosConfig.from_dict(meta["cfg"])
    case = next(c for c in meta["cases"] if c["tag"] == tag)
    om = OracleZonos(cfg, synthetic_weights(cfg, **case["model_kw"]))
    prefix = t.get(tag + "/prefix")
    raw = []
    torch.set_num_threads(4)
    ref = om.generate(t[tag + "/cond"], prefix, max_new_tokens=case["n"], sampling_params=case["params"],
                      raw_trace=raw)
    # (on this host's CPU the trajectory may differ from the fixture's near-ties; the check below
    # needs only the oracle's own logits and frames, and the case keeps its character)
    assert (ref.shape[-1] < case["n"]) == tag.startswith("greedy_eos"), ref.shape
    ref_delayed = om.last_delayed[0]

    lib, sp = L.lib(), torch.cuda.current_stream().cuda_stream
    p = 0 if prefix is None else prefix.shape[-1]
    total = p + case["n"] + 9
    tcap = total + 8
    st = {k: torch.zeros(1, dtype=torch.int32, device=DEV) for k in
          ("active", "pos", "offset", "remaining", "stopping", "step", "total_len")}
    delayed = torch.full((1, 9, tcap), 1025, dtype=torch.int32, device=DEV)
    prm = torch.tensor(bytearray(SamplingParams(temperature=0.0, cfg_scale=1.0).to_c()), dtype=torch.uint8).to(DEV)
    sl = L.Slots(*(st[k].data_ptr() for k in ("active", "pos", "offset", "remaining", "stopping", "step")),
                 delayed.data_ptr(), prm.data_ptr(), st["total_len"].data_ptr(), tcap, 1)
    pr = torch.zeros(9, max(p, 1), dtype=torch.int32, device=DEV)
    if p:
        pr[:, :p] = prefix[0].to(DEV, torch.int32)
    L.check(lib.zmi_delay_init(ctypes.byref(sl), 0, pr.data_ptr(), p, total, sp))
    for k, v in {"active": 1, "pos": 1, "offset": p, "remaining": case["n"] + 8, "total_len": total}.items():
        st[k][0] = v
    nxt = torch.zeros(1, 9, dtype=torch.int32, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int32, device=DEV)
    rows = torch.zeros(2, 9, 1026, device=DEV)  # cond row = the reference's logits, uncond row = 0, cfg 1
    for i, lg in enumerate(raw):
        assert int(st["active"][0]) == 1, f"stopped after {i} of {len(raw)} sampling calls"
        rows[0] = lg[0].to(DEV)
        if greedy_kernel and i > 0:
            L.check(lib.zmi_sample_step_greedy(ctypes.byref(sl), rows.data_ptr(), nxt.data_ptr(), 0, 1, None, 0,
                                               None, None, None, sp))
        else:
            L.check(lib.zmi_sample_step(ctypes.byref(sl), rows.data_ptr(), None, nxt.data_ptr(), cnt.data_ptr(),
                                        1 if i == 0 else 0, 0, 1, None, 0, None, None, None, sp))
        torch.cuda.synchronize()
    assert int(st["active"][0]) == 0, "the reference loop ended here"
    assert torch.equal(delayed[0, :, :total].cpu().long(), ref_delayed[:, :total]), tag
    off = int(st["offset"][0])
    k = off - 9
    n_audio = total - 9
    t_out = min(k, n_audio) if k >= 0 else max(n_audio + k, 0)
    out = torch.zeros(9, max(t_out, 1), dtype=torch.int64, device=DEV)
    if t_out:
        L.check(lib.zmi_delay_revert(ctypes.byref(sl), 0, out.data_ptr(), t_out, sp))
    torch.cuda.synchronize()
    assert torch.equal(out[:, :t_out].cpu().unsqueeze(0), ref), tag
