"""Static task plan of the persistent decode-step kernel (csrc/zmi_step.hip).

The kernel runs one 1024-thread workgroup per CU. Waves 0..14 of workgroup b walk the list
`layer pattern x n_layer + heads pattern` of b, wave w taking entries w, w + 15, ...; each entry
is one weight-slice task (reference ops it replaces: zonos/backbone/_torch.py:99-152 per layer,
zonos/model.py:100-116 for the heads). This module builds those lists on the host and checks,
by simulation, that every schedule it emits completes (no wave can wait on work queued behind
itself): the same check runs in the CPU test suite.

Task word: type | part << 3 | group << 7 | slot << 20 (slot = LDS reduction slot, or the CU's
member index inside its attention unit for ATT tasks).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

T_QKV, T_ATT, T_OUT, T_FC1, T_FC2, T_HEADS = range(6)
NAMES = {T_QKV: "qkv", T_ATT: "att", T_OUT: "out", T_FC1: "fc1", T_FC2: "fc2", T_HEADS: "heads"}
# (parts W of K per 8-column group) = zmi_gemv8's shape8 for each projection
PARTS = {T_QKV: 2, T_OUT: 4, T_FC1: 2, T_FC2: 8, T_HEADS: 2}
NCW = 15          # task waves per workgroup (wave 15 stages LayerNorm rows)
NSLOT = 32        # LDS reduction slots per workgroup
HKV = 4


def word(t: int, part: int, group: int, slot: int) -> int:
    assert 0 <= part < 16 and 0 <= group < 8192 and 0 <= slot < 256
    return t | (part << 3) | (group << 7) | (slot << 20)


def unpack(w: int) -> tuple[int, int, int, int]:
    return w & 7, (w >> 3) & 15, (w >> 7) & 8191, (w >> 20) & 255


@dataclass
class StepPlan:
    n_blocks: int
    rows: int
    att_cus: int
    tasks: np.ndarray       # uint32, all lists back to back
    hdr: np.ndarray         # int32 [n_blocks][4] = layer_off, layer_len, head_off, head_len
    groups: dict            # task type -> number of 8-column groups

    def layer_list(self, b: int) -> list[int]:
        o, n = int(self.hdr[b, 0]), int(self.hdr[b, 1])
        return [int(x) for x in self.tasks[o:o + n]]

    def head_list(self, b: int) -> list[int]:
        o, n = int(self.hdr[b, 2]), int(self.hdr[b, 3])
        return [int(x) for x in self.tasks[o:o + n]]


def build(n_blocks: int, rows: int, qkv_cols: int = 3072, d: int = 2048, ffn: int = 8192,
          head_cols: int = 9248) -> StepPlan:
    """Round-robin the 8-column groups of every projection over the workgroups (group g on
    workgroup g % n_blocks), all parts of a group on one workgroup (they combine in its LDS),
    and the attention units (row, kv head) over the workgroups modulo: workgroup b is member
    b // units of unit b % units, so a unit's members share b % 8 (one XCD under the observed
    round-robin placement; speed only)."""
    units = rows * HKV
    if n_blocks % units:
        raise ValueError(f"{n_blocks} workgroups do not split into {units} attention units")
    att_cus = n_blocks // units
    if att_cus not in (8, 16, 32, 64):
        raise ValueError(f"{att_cus} CUs per attention unit (need 8, 16, 32 or 64)")
    groups = {T_QKV: qkv_cols // 8, T_OUT: d // 8, T_FC1: 2 * ffn // 8, T_FC2: d // 8, T_HEADS: head_cols // 8}
    slot_base, nxt = {}, 0
    for t in (T_QKV, T_OUT, T_FC1, T_FC2, T_HEADS):
        slot_base[t] = nxt
        nxt += -(-groups[t] // n_blocks)
    if nxt > NSLOT:
        raise ValueError(f"plan needs {nxt} LDS reduction slots (> {NSLOT})")
    words, hdr = [], np.zeros((n_blocks, 4), np.int32)

    def gemv(t, b, out):
        for i, g in enumerate(range(b, groups[t], n_blocks)):
            for part in range(PARTS[t]):
                out.append(word(t, part, g, slot_base[t] + i))

    for b in range(n_blocks):
        lay = []
        gemv(T_QKV, b, lay)
        lay.append(word(T_ATT, 0, b % units, b // units))
        for t in (T_OUT, T_FC1, T_FC2):
            gemv(t, b, lay)
        head = []
        gemv(T_HEADS, b, head)
        hdr[b] = (len(words), len(lay), len(words) + len(lay), len(head))
        words += lay + head
    return StepPlan(n_blocks, rows, att_cus, np.array(words, np.uint32), hdr, groups)


def simulate(plan: StepPlan, n_layer: int) -> int:
    """Abstract execution of the plan: returns the number of scheduling rounds to completion, or
    raises if some state makes no progress (a wave waiting on work that can never run).

    Dependencies (the kernel's waits): QKV(l) and FC1(l) need their LayerNorm rows, staged by the
    workgroup's stager once FC2(l-1) (resp. OUT(l)) is complete everywhere; ATT(l) needs QKV(l)
    complete, publishes its partial, then needs every member of its unit published; OUT(l) needs
    every ATT(l) merged; FC2(l) needs FC1(l); HEADS needs FC2(L-1). A group completes when all its
    parts have run.
    """
    nb, units = plan.n_blocks, plan.rows * HKV
    seqs = []
    for b in range(nb):
        lay, head = plan.layer_list(b), plan.head_list(b)
        seqs.append([(l, w) for l in range(n_layer) for w in lay] + [(n_layer, w) for w in head])
    done_parts = {}       # (l, type, group) -> parts done
    groups_done = {}      # (l, type) -> groups complete
    att_pub, att_merged = {}, {}  # (l, unit) -> members published / merged
    pos = [[w for w in range(NCW)] for _ in range(nb)]   # next flattened index per wave
    att_stage = set()     # (b, l) once published (waiting for the merge)

    def complete(l, t):
        return groups_done.get((l, t), 0) == plan.groups[t]

    def ready(l, t):
        if t == T_QKV:
            return l == 0 or complete(l - 1, T_FC2)
        if t == T_ATT:
            return complete(l, T_QKV)
        if t == T_OUT:
            return sum(att_merged.get((l, u), 0) for u in range(units)) == nb
        if t == T_FC1:
            return complete(l, T_OUT)
        if t == T_FC2:
            return complete(l, T_FC1)
        return complete(n_layer - 1, T_FC2)

    rounds = 0
    while True:
        progress, remaining = False, False
        for b in range(nb):
            for w in range(NCW):
                i = pos[b][w]
                if i >= len(seqs[b]):
                    continue
                remaining = True
                l, wd = seqs[b][i]
                t, part, grp, slot = unpack(wd)
                if t == T_ATT:
                    if (b, l) not in att_stage:
                        if not ready(l, t):
                            continue
                        att_stage.add((b, l))
                        att_pub[(l, grp)] = att_pub.get((l, grp), 0) + 1
                        progress = True
                    if att_pub.get((l, grp), 0) < plan.att_cus:
                        continue
                    att_merged[(l, grp)] = att_merged.get((l, grp), 0) + 1
                else:
                    if not ready(l, t):
                        continue
                    k = (l, t, grp)
                    done_parts[k] = done_parts.get(k, 0) + 1
                    if done_parts[k] == PARTS[t]:
                        groups_done[(l, t)] = groups_done.get((l, t), 0) + 1
                pos[b][w] = i + NCW
                progress = True
        rounds += 1
        if not remaining:
            return rounds
        if not progress:
            raise RuntimeError(f"step plan deadlocks after {rounds} rounds")
