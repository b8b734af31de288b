"""CPU checks of the bench helpers (bench/bench_mine.py)."""


def test_sampled_supports_check_detects_a_wrong_count():
    """bench_mine.sampled_supports_ok (config 3's verification) recounts sampled itemsets on
    the host: the CPU miner's trie passes, a trie with one support changed fails."""
    import numpy as np
    from kubernetes_machine_learning_server_amd.bench.bench_mine import sampled_supports_ok
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.load()
    tx = generate("ds2_weak", seed=1)
    r = N.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.02)
    trie = {k: np.asarray(r[k]) for k in ("parent", "item", "count", "depth")}
    assert sampled_supports_ok(trie, tx.tx_ptr, tx.items, 1, 0, k=400)
    bad = dict(trie)
    bad["count"] = trie["count"].astype(np.int64) + (trie["depth"] >= 2)
    assert not sampled_supports_ok(bad, tx.tx_ptr, tx.items, 1, 0, k=400)
