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


def test_config5_pvc_alt_index_is_the_higher_support_rule_map(tmp_path):
    """bench.py's config-5 serving PVC: rules_alt.idx (the reload target) must be exactly the
    rule map of the same data at the higher support: pair rows filtered to counts >= the alt
    threshold, keys = the items frequent at it."""
    import numpy as np
    from kubernetes_machine_learning_server_amd.bench.bench_large import write_config5_pvc
    from kubernetes_machine_learning_server_amd.serve.index import RuleIndexData
    rng = np.random.default_rng(0)
    T, I = 1000, 50
    ids = np.array([1, 4, 7, 9, 20, 33], np.int64)
    fc = np.array([90, 40, 60, 31, 45, 30], np.int64)
    rows = {int(i): [] for i in range(I)}
    for a in range(len(ids)):
        for b in range(len(ids)):
            if a != b and rng.random() < 0.7:
                rows[int(ids[a])].append((int(ids[b]), int(rng.integers(10, min(fc[a], fc[b]) + 1))))
    row_ptr = [0]
    cons, cnt = [], []
    for i in range(I):
        rr = sorted(rows[i], key=lambda x: (-x[1], x[0]))
        cons += [c for c, _ in rr]
        cnt += [n for _, n in rr]
        row_ptr.append(len(cons))
    r = {"row_ptr": np.array(row_ptr, np.int64), "cons": np.array(cons, np.int32),
         "count": np.array(cnt, np.uint32)}
    info = write_config5_pvc(str(tmp_path), r, I, ids, fc, T, 30, alt_factor=1.5)
    alt = RuleIndexData.load(tmp_path / "rules_alt.idx")
    main = RuleIndexData.load(tmp_path / "api-data" / "pickles" / "rules.idx")
    assert info["alt_min_count"] == 45
    assert set(np.flatnonzero(alt.is_key)) == {1, 7, 20}
    assert set(np.flatnonzero(main.is_key)) == set(ids.tolist())
    for i in range(I):
        want = [(c, n) for c, n in sorted(rows[i], key=lambda x: (-x[1], x[0])) if n >= 45]
        got_c = alt.cons[alt.row_ptr[i]:alt.row_ptr[i + 1]].tolist()
        got_n = np.rint(alt.score[alt.row_ptr[i]:alt.row_ptr[i + 1]] * T).astype(int).tolist()
        assert list(zip(got_c, got_n)) == want
    assert (tmp_path / "api-data" / "pickles" / "best_tracks.pickle").exists()
    assert (tmp_path / "api-data" / "last_execution.txt").read_text() == "initial"
