"""GPU parity of the count-only deep miner (kernels/deep.hip) against the CPU count miner.

Every case compares the per-size itemset counts AND the content digest (the multiset hash of
every (itemset, support) pair, kmls/digest.hpp) with ``mine_cpu_count``, which is itself checked
against ``trie_digest`` of the full CPU trie (and so against the mlxtend-faithful oracle, via
test_miner_cpu.py).  Small step budgets force many spills (in-launch work stealing, the default,
or spill rounds); rank splits are combined by
hand (sum of counts and digest sums, xor of digest xors) and must equal the single-rank run.
"""
import numpy as np
import pytest

from kubernetes_machine_learning_server_amd.data.synthetic import generate

pytestmark = pytest.mark.gpu


def _cpu(N, tx, ms, max_len=0):
    return N.mine_cpu_count(tx.tx_ptr, tx.items, tx.n_items, ms, max_len)


def _gpu_miner(N, tx):
    g = N.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    return g


def _levels(per):
    per = list(per)
    while len(per) > 2 and per[-1] == 0:
        per.pop()
    return [int(x) for x in per[1:]]


def _same(d, c):
    assert _levels(d["per_level"]) == _levels(c["per_level"]), (d["per_level"], c["per_level"])
    assert d["n_itemsets"] == c["n_itemsets"]
    assert d["digest"] == c["digest"]


@pytest.mark.parametrize("shape,ms,n_tx", [("ds1", 0.05, None), ("ds1", 0.04, None),
                                             ("ds1", 0.03, None), ("tiny", 0.02, None),
                                             ("tiny", 0.01, 4000), ("ds_dense", 0.05, None)])
def test_deep_matches_cpu_count(gpu_mod, shape, ms, n_tx):
    tx = generate(shape, seed=0, **({"n_tx": n_tx} if n_tx else {}))
    g = _gpu_miner(gpu_mod, tx)
    d = g.mine_deep(ms)
    _same(d, _cpu(gpu_mod, tx, ms))


def test_deep_equals_full_trie_digest(gpu_mod):
    """The count-only digest is the digest of the complete trie (not just of another counter)."""
    tx = generate("ds1", seed=0)
    r = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.05)
    t = gpu_mod.trie_digest(r["parent"], r["item"], r["count"], r["depth"])
    d = _gpu_miner(gpu_mod, tx).mine_deep(0.05)
    assert d["digest"] == t["digest"]
    assert _levels(d["per_level"]) == [int(x) for x in t["per_depth"][1:]]


@pytest.mark.parametrize("budget0,budget,split_min", [(1, 1, 2), (2, 3, 64), (1, 8, 4)])
def test_deep_spill_rounds(gpu_mod, budget0, budget, split_min):
    """Spill rounds (steal off), tiny step budgets: every task spills, dense subtrees go through
    many rounds."""
    tx = generate("ds1", seed=0)
    d = _gpu_miner(gpu_mod, tx).mine_deep(0.04, budget0=budget0, budget=budget,
                                          split_min=split_min, steal=False)
    assert len(d["round_tasks"]) >= 2
    _same(d, _cpu(gpu_mod, tx, 0.04))


@pytest.mark.parametrize("budget,split_min,steal_idle", [(1, 2, 0), (3, 64, 0), (8, 4, 1),
                                                         (64, 8, 1), (2, 8, 2), (256, 8, 1)])
def test_deep_work_stealing(gpu_mod, budget, split_min, steal_idle):
    """One launch; waves that run dry ask busy waves for work.  steal_idle 1: direct hand-offs
    to the asking wave's inbox (the default); 0: the bottom frame to the shared queue at every
    check (tens of thousands of hand-offs through the ready flags); 2: a hand-off to the
    partner wave whenever it waits."""
    tx = generate("ds1", seed=0)
    d = _gpu_miner(gpu_mod, tx).mine_deep(0.04, budget=budget, split_min=split_min,
                                          steal=True, steal_idle=steal_idle)
    # one stealing launch (after the pre-split launch of the heaviest tasks, when any)
    assert len(d["round_tasks"]) == 1 + (d["presplit"][0] > 0)
    if steal_idle == 0:
        assert d["spilled_tasks"] > 0
    elif budget <= 64:  # (at 256 passes between checks this small problem needs no hand-off)
        assert d["handoffs"] > 0, d
    _same(d, _cpu(gpu_mod, tx, 0.04))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_deep_rank_split_combines(gpu_mod, world):
    tx = generate("ds1", seed=0)
    g = _gpu_miner(gpu_mod, tx)
    ref = g.mine_deep(0.04)
    per = np.zeros(64, dtype=np.uint64)
    dsum, dxor = 0, 0
    for r in range(world):
        d = g.mine_deep(0.04, rank=r, world=world)
        p = np.array(d["per_level"], dtype=np.uint64)
        per[:len(p)] += p
        dsum = (dsum + int(d["digest"][:16], 16)) % (1 << 64)
        dxor ^= int(d["digest"][16:], 16)
    assert _levels(per) == _levels(ref["per_level"])
    assert f"{dsum:016x}{dxor:016x}" == ref["digest"]


@pytest.mark.parametrize("max_len", [2, 3, 5])
def test_deep_max_len(gpu_mod, max_len):
    tx = generate("ds1", seed=0)
    d = _gpu_miner(gpu_mod, tx).mine_deep(0.03, max_len=max_len)
    _same(d, _cpu(gpu_mod, tx, 0.03, max_len))


def test_deep_small_stack_spills(gpu_mod):
    """A stack too small for deep recursion spills instead of overflowing."""
    tx = generate("ds1", seed=0)
    d = _gpu_miner(gpu_mod, tx).mine_deep(0.04, stack_mb=1, blocks_per_cu=1)
    _same(d, _cpu(gpu_mod, tx, 0.04))


def _arena_trie(arena):
    """The downloaded node arena (ids in allocation order, size 0 = unused id) as a trie whose
    parents come first: nodes sorted by size, parent ids remapped."""
    dep = np.asarray(arena["depth"])
    keep = np.flatnonzero(dep > 0)
    order = keep[np.argsort(dep[keep], kind="stable")]
    new_id = np.full(len(dep), -1, np.int64)
    new_id[order] = np.arange(len(order))
    par = np.asarray(arena["parent"])[order]
    par = np.where(par >= 0, new_id[np.maximum(par, 0)], -1)
    return (par, np.asarray(arena["item"])[order], np.asarray(arena["count"])[order],
            dep[order])


@pytest.mark.parametrize("ms,world", [(0.05, 1), (0.04, 1), (0.04, 3)])
def test_deep_emit_arena_is_the_trie(gpu_mod, ms, world):
    """Emit mode: every frequent itemset becomes a node of the HBM trie arena.  The downloaded
    arena, as a trie, has the CPU miner's trie digest (every itemset and support, nothing
    else), and the device's own arena digest equals it; the count-only digest is unchanged.
    Rank splits: each rank's arena holds its share (sizes >= 3 past rank 0)."""
    tx = generate("ds1", seed=0)
    g = _gpu_miner(gpu_mod, tx)
    ref = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms)
    want = gpu_mod.trie_digest(ref["parent"], ref["item"], ref["count"], ref["depth"])
    s, x, per = 0, 0, np.zeros(64, np.int64)
    for rank in range(world):
        d = g.mine_deep(ms, rank=rank, world=world, emit=True, budget=4)
        assert d["arena_nodes"] <= d["arena_cap"]
        dev = g.deep_arena_digest(1 if rank == 0 else 3)
        a = g.deep_arena_download(d["arena_nodes"])
        par, item, cnt, dep = _arena_trie(a)
        # (every rank's arena holds the root levels as parents; sizes 1-2 count on rank 0)
        host = gpu_mod.trie_digest(par, item, cnt, dep, 1 if rank == 0 else 3)
        assert host["digest"] == dev["digest"], (rank, host, dev)
        s = (s + int(dev["sum"])) % (1 << 64)
        x ^= int(dev["xor"])
        per[:len(dev["per_depth"])] += np.asarray(dev["per_depth"], np.int64)
        if world == 1:
            assert d["digest"] == want["digest"]
    assert f"{s:016x}{x:016x}" == want["digest"]
    assert [int(v) for v in per[1:len(want["per_depth"])]] == [int(v) for v in want["per_depth"][1:]]
