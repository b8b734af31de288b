"""CPU checks of the deep miner's host-side combine and of the full-mining estimator
(parallel/deep.py): the per-rank partials combine into the whole-problem result, and the
sampled-virtual-rank estimate is exact with zero error when every rank is sampled and unbiased
over many draws."""
import random

import pytest

from kubernetes_machine_learning_server_amd.parallel.deep import combine_partials, estimate_total


class FakeDeep:
    """mine_deep over a fixed population of per-rank per-size counts (heavy-tailed)."""

    def __init__(self, world: int, seed: int = 1, tail: int = 50):
        rng = random.Random(seed)
        self.world = world
        self.parts = []
        for r in range(world):
            heavy = tail if rng.random() < 0.05 else 1
            per = [0, 0, 0] + [heavy * rng.randint(1, 1000) * (d + 1) for d in range(6)]
            self.parts.append(per)
        self.calls = []

    def mine_deep(self, ms, max_len, rank, world, comm, **opts):
        assert world == self.world and comm is None
        self.calls.append(rank)
        per = self.parts[rank]
        return {"per_level": per, "n_itemsets": sum(per[1:]), "digest": "0" * 32,
                "candidates": 0}

    def total(self):
        return sum(sum(p[1:]) for p in self.parts)


def test_estimate_exact_when_every_rank_is_sampled():
    g = FakeDeep(16)
    e = estimate_total(g, 0.01, 16, 16)
    assert sorted(g.calls) == list(range(16))
    assert e["n_itemsets_estimate"] == g.total()
    assert e["n_itemsets_se"] == 0  # finite-population correction: nothing left unsampled
    for row in e["per_size"]:
        assert row["estimate"] == sum(p[row["size"]] for p in g.parts)


@pytest.mark.parametrize("tail,min_cover", [(50, None), (1, 0.9)])
def test_estimate_unbiased_and_se_calibrated(tail, min_cover):
    """Unbiased whatever the tail; the sample-variance error bar is calibrated without a heavy
    tail (with a 50x heavy tail and 20 samples it undercovers, as sample variances of heavy-tailed
    populations do — the full-count partials, not the estimate, are config 2's result)."""
    g = FakeDeep(200, seed=3, tail=tail)
    exact = g.total()
    ests, covered = [], 0
    for s in range(400):
        e = estimate_total(g, 0.01, 200, 20, seed=s)
        ests.append(e["n_itemsets_estimate"])
        covered += abs(e["n_itemsets_estimate"] - exact) <= 2.5 * e["n_itemsets_se"]
    mean = sum(ests) / len(ests)
    assert abs(mean - exact) / exact < 0.05
    if min_cover is not None:
        assert covered / len(ests) > min_cover


def test_estimate_budget_stops_after_two_samples():
    g = FakeDeep(64)
    e = estimate_total(g, 0.01, 64, 30, budget_s=1e-9)
    assert e["samples"] == 2 and len(g.calls) == 2


def test_combine_partials_sums_counts_and_digest_terms():
    parts = [{"per_level": [0, 3, 2], "digest": f"{1:016x}{5:016x}", "candidates": 7},
             {"per_level": [0, 1, 0, 4], "digest": f"{(1 << 64) - 1:016x}{3:016x}",
              "candidates": 1}]
    d = combine_partials(parts)
    assert d["per_level"] == [0, 4, 2, 4] and d["n_itemsets"] == 10 and d["max_depth"] == 3
    assert d["digest"] == f"{0:016x}{5 ^ 3:016x}"  # sums wrap mod 2^64, xors combine
    assert d["candidates"] == 8


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
