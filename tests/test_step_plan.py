"""Host-side checks of the persistent decode-step plan (zonos_vibes_amd/step_plan.py): every
projection group is scheduled exactly once with all its K parts on one workgroup, LDS slots are in
range and unique per group, attention units have all their members, and the static schedule
completes (no wave waits on work queued behind itself)."""
import pytest

from zonos_vibes_amd import step_plan as sp


@pytest.mark.parametrize("nb,rows", [(256, 2), (256, 4), (512, 2), (512, 4)])
def test_plan_covers_every_group_once(nb, rows):
    p = sp.build(nb, rows)
    owner, slot_of = {}, {}
    att = {}
    for b in range(nb):
        for w in p.layer_list(b) + p.head_list(b):
            t, part, g, slot = sp.unpack(w)
            if t == sp.T_ATT:
                assert (g, slot) not in att
                att[(g, slot)] = b
                continue
            assert (t, g, part) not in owner
            owner[(t, g, part)] = b
            assert 0 <= slot < sp.NSLOT
            assert slot_of.setdefault((b, t, g), slot) == slot
    for t, n in p.groups.items():
        for g in range(n):
            assert len({owner[(t, g, part)] for part in range(sp.PARTS[t])}) == 1
    # a slot is never shared by two groups of one workgroup
    seen = {}
    for (b, t, g), slot in slot_of.items():
        assert seen.setdefault((b, slot), (t, g)) == (t, g)
    units = rows * sp.HKV
    assert sorted(att) == [(u, j) for u in range(units) for j in range(p.att_cus)]
    assert all(b % units == u for (u, j), b in att.items())


@pytest.mark.parametrize("n_layer", [1, 2, 26])
def test_plan_schedule_completes(n_layer):
    assert sp.simulate(sp.build(256, 2), n_layer) > 0


def test_plan_rejects_bad_geometry():
    with pytest.raises(ValueError):
        sp.build(250, 2)
    with pytest.raises(ValueError):
        sp.build(1024, 2)   # 128 CUs per attention unit
    with pytest.raises(ValueError):
        sp.build(128, 2)    # 40 LDS reduction slots per workgroup


def test_word_roundtrip():
    for args in [(0, 0, 0, 0), (5, 15, 8191, 255), (3, 1, 2047, 10)]:
        assert sp.unpack(sp.word(*args)) == args
