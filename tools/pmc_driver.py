"""Short drivers for rocprofv3 counter passes (a --pmc pass serialises every dispatch, so only the
kernel under study runs): the fc1 GEMV of all 26 layers, or the attention of all 26 layers at the
C2 mean position, on the synthetic Zonos-v0.1 engine (B = 1, two CFG rows).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fc1 -o pmc -- \
        python tools/pmc_driver.py fc1
    rocprofv3 --pmc FETCH_SIZE ... -- python tools/pmc_driver.py attn        (and WRITE_SIZE)
    rocprofv3 --pmc FETCH_SIZE ... -- python tools/pmc_driver.py attnblk     (fused QKV + attention + out_proj)
    rocprofv3 --pmc FETCH_SIZE ... -- python tools/pmc_driver.py fc2         (the fc2 GEMV)
    rocprofv3 --pmc SQ_LDS_BANK_CONFLICT ... -- python tools/pmc_driver.py step   (the whole default decode step)
then tools/pmc_summary.py turns the counter CSV into the per-launch JSON kept under profiles/.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402

POS = 591


def main(which: str, reps: int = 2):
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=POS + 64, max_prefill=16)
    e = m.engine
    with torch.cuda.stream(e.stream):
        e.row_pos[:2] = POS
        e.row_kv[:2] = torch.arange(2, dtype=torch.int32, device=dev)
        e.x.normal_()
        e.q.normal_()
        e.kc.normal_()
        e.vc.normal_()
    e.stream.synchronize()
    e.pos_hi[0] = POS
    plan = e._plan(2, e._segments(1, 1)[0][1])  # the form the decode step uses at POS
    for _ in range(reps):
        if which in ("fc1", "fc2"):
            for kind, it in plan:
                if kind == "gemv" and ((it[1] == _lib.EPI_SWIGLU) if which == "fc1" else
                                       (it[1] == _lib.EPI_RESIDUAL and it[0].K == e.F)):
                    e._run_gemv(it)
        elif which == "attn":
            for i in range(e.L):
                e._attention(i, e.q, 2, None, e.row_pos, e.smax - 1, e.attn)
        elif which == "attnblk":  # the fused QKV + attention launch of every layer (granules fresh per rep)
            e.blk_gran.zero_()
            for kind, it in plan:
                if kind == "attnblk":
                    e._run_attn_block(it)
        elif which == "step":  # the whole C2 decode step (launch plan + sampler) at POS, position held
            e.enqueue_step(form=e._segments(1, 1)[0][1])
        else:
            raise SystemExit(f"unknown driver {which}")
    e.stream.synchronize()
    e.check_errors()
    print(f"{which}: {reps} x {e.L} launches at position {POS}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "fc1")
