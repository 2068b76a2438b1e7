"""Does the placement of one engine buffer set the C2 step time? Each buffer is swapped for a copy at a new
address (behind a spacer allocation), the plan rebuilt and the step timed, then swapped back (one JSON line
per measurement)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402

NAMES = ["x", "q", "attn", "xn", "h", "logits", "row_kv", "row_pos", "blk_gran", "blk_err", "attn_work", "kc", "vc",
         "weights"]


def main():
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=bench.LC + bench.N_NEW + 9,
                        max_prefill=bench.LC + 1)
    e = m.engine
    cond = bench.cond_tensor(0, e.d, dev)
    keep = []

    def t(label, name):
        e._build_plan()
        us, _ = bench.time_decode_step(m, cond, steps=128)
        print(json.dumps(dict(case=label, buf=name, us=round(us, 1))), flush=True)

    def clone_w(w):
        if isinstance(w, torch.Tensor):
            return w.clone()
        if isinstance(w, dict):
            return {k: clone_w(v) for k, v in w.items()}
        if isinstance(w, list):
            return [clone_w(v) for v in w]
        return w

    t("base", "-")
    for rep in range(2):
        for name in NAMES:
            keep.append(torch.empty(int(torch.randint(1, 1 << 20, (1,))) * 256, dtype=torch.uint8, device=dev))
            old = getattr(e, name) if name != "weights" else e.w
            new = clone_w(old)
            if name == "weights":
                e.w = new
            else:
                setattr(e, name, new)
            t("swapped", name)
            if name == "weights":
                e.w = old
            else:
                setattr(e, name, old)
            del new
            t("restored", name)


if __name__ == "__main__":
    main()
