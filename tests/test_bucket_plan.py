"""Readiness-aware gradient bucket plan (SURVEY.md §5.8 overlap analysis; replaces the
reference's one blocking exchange after backward, ref.py:264,396)."""
import torch

from ddlpc.config import ModelConfig
from ddlpc.models import UNet
from ddlpc.parallel import GradBucketReducer
from ddlpc.parallel.bucket_plan import (XGMI_LAT_US, XGMI_RING_GBPS, backward_readiness,
                                        evaluate_cuts, plan_buckets, plan_for_model,
                                        size_plan_cuts)
from ddlpc.parallel.flat import flatten_module


def _setup(mc=None):
    mc = mc or ModelConfig(out_classes=6)
    m = UNet.from_config(mc)
    fl = flatten_module(m)
    names = {id(p): n for n, p in m.named_parameters()}
    ready = backward_readiness(mc, 256, [names[id(p)] for p in fl.order])
    return mc, m, fl, names, ready


def test_readiness_is_backward_order():
    """The flat order is backward order: readiness never decreases along it; the head is
    ready first, the first encoder conv last; the high-resolution encoder (down_conv1..3)
    holds a small share of the bytes but a large share of backward compute."""
    mc, m, fl, names, ready = _setup()
    assert all(b >= a - 1e-12 for a, b in zip(ready[:-1], ready[1:]))
    assert names[id(fl.order[0])].startswith("conv_last") and ready[-1] == 1.0
    assert names[id(fl.order[-1])].startswith("down_conv1.")
    hi = [i for i, p in enumerate(fl.order) if names[id(p)].split(".")[0] in
          ("down_conv1", "down_conv2", "down_conv3")]
    total = sum(p.numel() for p in fl.order)
    share = sum(fl.order[i].numel() for i in hi) / total
    assert share < 0.12, share
    assert ready[hi[0] - 1] < 0.85        # ... while >= 15% of backward is still to run


def test_plan_closes_a_bucket_at_the_high_resolution_boundary():
    """Flagship config (256², width/2, batch 256, 8 ranks over xGMI): every bucket but a
    tiny tail finishes before backward ends, and the plan beats the size-only cut."""
    mc, m, fl, names, ready = _setup()
    plan = plan_for_model(m, fl.order, mc, 256, 256, 8, "nccl", 8.0)
    nb = [p.numel() * 4.0 for p in fl.order]
    assert plan.cuts[0] == 0 and plan.cuts[-1] == len(fl.order)
    assert 3 <= len(plan.cuts) - 1 <= 16
    assert all(t < plan.backward_ms for t in plan.bucket_done_ms[:-1])
    tail = sum(nb[plan.cuts[-2]:])
    assert tail <= 0.02 * sum(nb), tail
    assert all(names[id(p)].split(".")[0] in ("down_conv1", "down_conv2")
               for p in fl.order[plan.cuts[-2]:])
    size = evaluate_cuts(size_plan_cuts(nb, 8 * 2**20), nb, ready, plan.backward_ms, 8,
                         XGMI_RING_GBPS, XGMI_LAT_US)
    assert plan.finish_ms < size.finish_ms and plan.exposed_ms < size.exposed_ms
    assert max(sum(nb[a:b]) for a, b in zip(plan.cuts[:-1], plan.cuts[1:])) <= 8 * 2**20


def test_plan_dp_is_optimal_on_small_cases():
    """Brute force over every contiguous partition of a small chain."""
    import itertools
    nb = [3e6, 1e6, 8e6, 2e6, 5e5, 4e6, 1e5]
    ready = [0.1, 0.2, 0.5, 0.6, 0.8, 0.9, 1.0]
    plan = plan_buckets(nb, ready, 5.0, 8, 100.0, 30.0, 1e9)
    best = None
    for r in range(0, len(nb)):
        for inner in itertools.combinations(range(1, len(nb)), r):
            cuts = [0, *inner, len(nb)]
            ev = evaluate_cuts(cuts, nb, ready, 5.0, 8, 100.0, 30.0)
            j = ev.finish_ms + 0.25 * 30e-3 * (len(cuts) - 1)
            best = j if best is None else min(best, j)
    got = plan.finish_ms + 0.25 * 30e-3 * (len(plan.cuts) - 1)
    assert abs(got - best) < 1e-9, (got, best)


def test_reducer_builds_buckets_from_cuts():
    mc, m, fl, names, ready = _setup(ModelConfig(out_classes=3, depth=4, width_divisor=8))
    cuts = [0, 5, 17, len(fl.order)]
    red = GradBucketReducer(fl, bucket_mb=1.0, cuts=cuts)
    assert len(red.buckets) == 3
    for b, (a, e) in zip(red.buckets, zip(cuts[:-1], cuts[1:])):
        assert b.params == fl.order[a:e]
        assert b.start == fl.span(fl.order[a])[0] and b.end == fl.span(fl.order[e - 1])[1]
    # every gradient element belongs to exactly one bucket (padding aside)
    cov = torch.zeros(fl.numel, dtype=torch.int32)
    for b in red.buckets:
        cov[b.start:b.end] += 1
    for p in fl.order:
        a, e = fl.span(p)
        assert bool((cov[a:e] == 1).all())
    import pytest
    with pytest.raises(ValueError):
        GradBucketReducer(fl, cuts=[0, 3, 3, len(fl.order)])
