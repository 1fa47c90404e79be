"""Side-branch planning (PlanOp::join): ResNet projection shortcuts run on a second stream beside
the unit's reduce/3x3 convs.  The arena must keep everything the branch touches disjoint from what
the concurrent ops write (CPU-only: checks the planner's buffer ranges)."""
import pytest


def _overlap(a, b):
    return a[0] < b[1] and b[0] < a[1]


def _check_branches(plan):
    ops = plan["ops"]
    branches = [(i, o["join"]) for i, o in enumerate(ops) if o["join"] >= 0]
    for i, j in branches:
        side = ops[i]["bufs"]
        assert j >= i + 2
        assert any(side["out"] == ops[j]["bufs"].get(r) for r in ("in", "in2", "in3")), "join consumes the branch"
        for k in range(i + 1, j):
            mid = ops[k]["bufs"]
            assert all(side["out"] != mid.get(r) for r in ("in", "in2", "in3")), "op inside the branch reads it"
            for wr in ("out", "out2", "out3"):  # concurrent writes never touch the branch's buffers
                if wr in mid:
                    for r, rng in side.items():
                        assert not _overlap(mid[wr], rng), (ops[k]["name"], wr, ops[i]["name"], r)
            for r, rng in mid.items():  # and the branch never writes what they touch
                assert not _overlap(side["out"], rng), (ops[i]["name"], ops[k]["name"], r)
    return branches


def test_resnet50_projection_shortcuts_are_branches(native, models):
    path, _, _ = models["get_rn50"]()
    plan = native.plan_summary(path, 32, side_branches=True)
    branches = _check_branches(plan)
    names = [plan["ops"][i]["name"] for i, _ in branches]
    assert len(branches) == 4, names  # one projection conv per stage
    for i, j in branches:
        # reduce, 3x3, then the expand conv joins; at the stage-1 -> stage-2 boundary the reduce conv
        # is inside the conv_pair before the branch, so only the 3x3 runs beside it
        assert plan["ops"][j]["residual"] and j in (i + 2, i + 3)
        if j == i + 2:
            assert plan["ops"][i - 1]["kind"] == "conv_pair" and plan["ops"][i - 1]["store_preact"]


@pytest.mark.parametrize("B", [1, 8])
def test_tiny_resnet_branches_safe(native, models, B):
    path, _, _ = models["tiny"]
    _check_branches(native.plan_summary(path, B, side_branches=True))


def test_vit_plan_branches_safe(native, models):
    path, _, _ = models["get_vit"]("tiny")
    _check_branches(native.plan_summary(path, 4, side_branches=True))


def test_no_branches_unless_asked(native, models):
    path, _, _ = models["get_rn50"]()
    assert all(o["join"] < 0 for o in native.plan_summary(path, 32)["ops"])
